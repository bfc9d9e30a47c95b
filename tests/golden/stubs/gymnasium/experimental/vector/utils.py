def batch_space(space, n=1):
    return space
