"""Reference scripts package (splendor_gym/scripts/): evaluation suite, game logger, random rollout.
Imported lazily by name; nothing here touches the GPU at import time."""
