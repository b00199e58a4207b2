"""herdsman_amd -- MI355X-native FHE ciphertext-op backend for herdsman.

The product is the C-ABI library ``herdsman_amd/lib/libherdsman_fhe.so``
(declared in ``include/plugins/fhe_backend.h``, kernels in
``herdsman_amd/csrc``).  ``herdsman_amd.backend`` is a thin ctypes binding used
by the tests and ``bench.py``; the production caller is the C++ GPU worker
group (``herdsman_amd/host``) that plugs into herdsman's IWorkerGroup seam.
"""
from .backend import (  # noqa: F401
    Context,
    FheBackendError,
    SCHEME_BFV,
    SCHEME_CKKS,
    library_path,
    load_library,
)
