"""gfx950 HIP kernels (built into ops/libthk.so by ops/build.py) and their autograd wrappers."""
