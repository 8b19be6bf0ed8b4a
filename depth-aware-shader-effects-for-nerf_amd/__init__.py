"""nerfmi — MI355X-native NeRF volumetric renderer (import name ``nerfmi``)."""
