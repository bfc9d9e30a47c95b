"""Minimal gymnasium 0.29 API stand-in used ONLY to import the reference's
PPO/A2C hot path in the survey container for golden-vector generation.
Not shipped, not imported by the product or by GPU tests."""
from . import spaces  # noqa: F401
from .spaces import Space  # noqa: F401


class Env:
    pass


class Wrapper(Env):
    def __init__(self, env):
        self.env = env


class ObservationWrapper(Wrapper):
    pass


class RewardWrapper(Wrapper):
    pass


class ActionWrapper(Wrapper):
    pass
