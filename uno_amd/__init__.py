"""uno_amd: MI355X-native sparse symmetric-indefinite KKT backend for Uno (amontoison/Uno).

The product is the C-ABI library uno_amd/libuno_kkt.so (include/uno_kkt.h) built from the HIP
sources in uno_amd/csrc; uno_amd.kkt is its ctypes binding plus Python mirrors of Uno's plugin
surface used by the tests and bench.py.
"""
from .kkt import (HipKKT, HipLDLSolver, KKTError, SparseSymmetricMatrix, UnstableRegularization,  # noqa: F401
                  arrowband, coo_symv, load_library, regularize_augmented_matrix, SEEDS,
                  LocalGroup, GlooComm, rccl_unique_id, debug_partition, debug_partition_gate)
