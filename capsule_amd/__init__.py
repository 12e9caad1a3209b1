"""capsule_amd — MI355X-native packet hot path of capsule-rs/capsule.

Batched Ethernet -> IPv4/IPv6 -> UDP/TCP parse, RFC 1071 Internet checksums,
5-tuple flow hash and the examples/nat64 6to4 rewrite as hand-written gfx950
HIP kernels behind the C ABI of include/capsule_gpu.h.  See DESIGN.md.
"""
from . import _native as native  # noqa: F401
from . import synth  # noqa: F401

__all__ = ["native", "synth", "packets"]


def __getattr__(name):
    # `packets` needs torch; import it lazily so synth/native stay light.
    if name in ("packets", "shards"):
        import importlib

        return importlib.import_module(f"{__name__}.{name}")
    raise AttributeError(name)
