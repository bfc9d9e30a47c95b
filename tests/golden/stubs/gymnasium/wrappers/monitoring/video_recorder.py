"""Import-only stub (gymnasium 0.29.1 is absent): the reference's vec_episode_recorder imports
VideoRecorder at module load; the golden scripts never record video."""


class VideoRecorder:
    def __init__(self, *a, **k):
        raise NotImplementedError("video recording is not available in the golden-vector harness")
