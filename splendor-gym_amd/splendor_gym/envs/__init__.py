from .splendor_env import SplendorEnv, make

__all__ = ["SplendorEnv", "make"]
