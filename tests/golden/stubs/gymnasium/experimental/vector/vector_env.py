from typing import Any

ArrayType = Any


class VectorEnv:
    num_envs: int
    single_observation_space = None
    single_action_space = None
    observation_space = None
    action_space = None

    @property
    def unwrapped(self):
        return self


class VectorWrapper(VectorEnv):
    def __init__(self, env):
        self.env = env

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self.env, name)

    @property
    def unwrapped(self):
        return self.env.unwrapped

    def reset(self, **kw):
        return self.env.reset(**kw)

    def step(self, actions):
        return self.env.step(actions)
