from .vector_env import VectorEnv, VectorWrapper  # noqa: F401
