"""rustfs_amd — MI355X-native Reed–Solomon erasure engine for the rustfs hot path.

The GPU work lives in ``librsgpu.so`` (HIP kernels for gfx950 behind the C ABI
in ``include/rsgpu.h``).  This package is the host-side mirror of the
reference's codec interface (``Erasure`` / ``ReedSolomonEncoder`` /
``HashAlgorithm`` / bitrot framing) used by the tests and the bench.
"""
from ._lib import (  # noqa: F401
    InvalidDataError,
    RsgError,
    RSG_HASH_HIGHWAY256S,
    RSG_HASH_HIGHWAY256S_LEGACY,
    RSG_HASH_NONE,
    RSG_RECONSTRUCT_DATA,
    RSG_RECONSTRUCT_MISSING,
    RSG_RECONSTRUCT_REENCODE_PARITY,
    device_count,
)
from .erasure import (  # noqa: F401
    Erasure,
    ErasureConstructionError,
    GpuCodecDecodeEngine,
    ReedSolomonEncoder,
    UnsupportedModernShardCount,
    ZeroBlockSize,
    ZeroDataShards,
    calc_shard_size,
    matrix,
)
