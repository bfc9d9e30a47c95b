import numpy as np


class Space:
    def __init__(self, shape=None, dtype=None):
        self._shape = None if shape is None else tuple(shape)
        self.dtype = None if dtype is None else np.dtype(dtype)

    @property
    def shape(self):
        return self._shape


class Box(Space):
    def __init__(self, low, high, shape=None, dtype=np.float32):
        if shape is None:
            shape = np.shape(low) if np.ndim(low) else np.shape(high)
        super().__init__(shape, dtype)
        self.low = np.broadcast_to(np.asarray(low, dtype=self.dtype), self.shape).copy()
        self.high = np.broadcast_to(np.asarray(high, dtype=self.dtype), self.shape).copy()

    def sample(self):
        if np.issubdtype(self.dtype, np.integer):
            return np.random.randint(self.low, self.high.astype(np.int64) + 1, size=self.shape).astype(self.dtype)
        lo = np.where(np.isfinite(self.low), self.low, -1.0)
        hi = np.where(np.isfinite(self.high), self.high, 1.0)
        return np.random.uniform(lo, hi, size=self.shape).astype(self.dtype)


class Discrete(Space):
    def __init__(self, n, start=0):
        super().__init__((), np.int64)
        self.n = int(n)
        self.start = start

    def sample(self):
        return np.int64(np.random.randint(self.n))


class MultiDiscrete(Space):
    def __init__(self, nvec, dtype=np.int64):
        self.nvec = np.asarray(nvec, dtype=np.int64)
        super().__init__(self.nvec.shape, dtype)


class Dict(Space):
    def __init__(self, spaces=None, **kw):
        super().__init__(None, None)
        self.spaces = dict(spaces or {}, **kw)

    def __getitem__(self, k):
        return self.spaces[k]

    def items(self):
        return self.spaces.items()


class Tuple(Space):
    def __init__(self, spaces):
        super().__init__(None, None)
        self.spaces = tuple(spaces)
