"""sfx -- MI355X-native successor-feature hot path (libsfx.so, gfx950 HIP kernels).

Import the engine lazily so ``sfx.build`` works on a machine without the built library.
"""
__all__ = ["SFEngine", "version"]


def __getattr__(name):
    if name == "SFEngine":
        from .engine import SFEngine
        return SFEngine
    if name == "version":
        from ._lib import version
        return version
    raise AttributeError(name)
