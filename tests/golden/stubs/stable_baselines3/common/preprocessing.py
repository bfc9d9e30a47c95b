import numpy as np


def get_flattened_obs_dim(space):
    return int(np.prod(space.shape))
