from typing import TypeVar

ObsType = TypeVar("ObsType")
ActType = TypeVar("ActType")
WrapperObsType = TypeVar("WrapperObsType")
WrapperActType = TypeVar("WrapperActType")
from . import Env, Wrapper  # noqa: E402,F401
