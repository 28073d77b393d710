"""gymnasium if installed, else a minimal stand-in with the same surface.

The reference requires gymnasium>=0.29.1 (pyproject.toml:14); this image has none, and the
package must import without it.  The stand-in covers what SplendorEnv, the
wrappers and the vector env use: Env (np_random seeding as in gymnasium 0.29), Wrapper,
spaces.Discrete, spaces.Box, spaces.MultiDiscrete.
"""
import numpy as np

try:  # pragma: no cover - depends on the environment
    import gymnasium as _gym

    Env = _gym.Env
    Wrapper = _gym.Wrapper
    spaces = _gym.spaces
    HAVE_GYMNASIUM = True
except ImportError:
    HAVE_GYMNASIUM = False

    class _Space:
        def seed(self, seed=None):
            self._rng = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
            return [seed]

        @property
        def np_random(self):
            if getattr(self, "_rng", None) is None:
                self.seed(None)
            return self._rng

    class Discrete(_Space):
        def __init__(self, n, seed=None, start=0):
            self.n, self.start, self.shape, self.dtype = int(n), int(start), (), np.dtype(np.int64)
            if seed is not None:
                self.seed(seed)

        def sample(self, mask=None):
            if mask is not None:
                legal = np.flatnonzero(mask)
                return int(self.start + (self.np_random.choice(legal) if len(legal) else 0))
            return int(self.start + self.np_random.integers(self.n))

        def contains(self, x):
            try:
                x = int(x)
            except (TypeError, ValueError):
                return False
            return self.start <= x < self.start + self.n

        def __repr__(self):
            return f"Discrete({self.n})"

    class Box(_Space):
        def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
            self.dtype = np.dtype(dtype)
            self.shape = tuple(shape) if shape is not None else np.shape(low)
            self.low = np.full(self.shape, low, dtype=self.dtype)
            self.high = np.full(self.shape, high, dtype=self.dtype)
            if seed is not None:
                self.seed(seed)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and np.can_cast(x.dtype, self.dtype) and bool(
                np.all(x >= self.low) and np.all(x <= self.high))

        def sample(self):
            return self.np_random.integers(self.low, self.high, endpoint=True, dtype=self.dtype)

        def __repr__(self):
            return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"

    class MultiDiscrete(_Space):
        def __init__(self, nvec, seed=None):
            self.nvec = np.asarray(nvec, dtype=np.int64)
            self.shape, self.dtype = self.nvec.shape, np.dtype(np.int64)

        def sample(self):
            return (self.np_random.random(self.nvec.shape) * self.nvec).astype(np.int64)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all((x >= 0) & (x < self.nvec)))

    class _Spaces:
        pass

    spaces = _Spaces()
    spaces.Discrete, spaces.Box, spaces.MultiDiscrete = Discrete, Box, MultiDiscrete

    class Env:
        metadata = {"render_modes": []}
        render_mode = None
        _np_random = None

        def reset(self, *, seed=None, options=None):
            if seed is not None:
                self._np_random = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))

        @property
        def np_random(self):
            if self._np_random is None:
                self._np_random = np.random.Generator(np.random.PCG64(np.random.SeedSequence(None)))
            return self._np_random

        @property
        def unwrapped(self):
            return self

        def close(self):
            pass

    class Wrapper(Env):
        """gymnasium.Wrapper surface the reference wrappers rely on: `env`, delegated reset /
        step / spaces / attributes (e.g. `state`), `unwrapped`."""

        def __init__(self, env):
            self.env = env

        def reset(self, **kwargs):
            return self.env.reset(**kwargs)

        def step(self, action):
            return self.env.step(action)

        def __getattr__(self, name):
            if name.startswith("_"):
                raise AttributeError(name)
            return getattr(self.env, name)

        @property
        def unwrapped(self):
            return self.env.unwrapped

        @property
        def np_random(self):
            return self.env.np_random

        def close(self):
            return self.env.close()
