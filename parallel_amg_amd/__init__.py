"""parallel_amg_amd — MI355X-native AMG V-cycle solve path (SPEC.md).

Host layer mirroring the PartitionedArrays.jl operator surface the reference builds on
(/root/reference/README.md:2) over the C-ABI library libpamg.so (include/pamg.h): HIP/gfx950
kernels for SpMV / residual / weighted Jacobi / restriction / prolongation, RCCL ghost
exchange, and a host smoothed-aggregation setup.
"""
from .backend import DistributedBackend, SequentialBackend  # noqa: F401
from .checkpoint import load_hierarchy, save_hierarchy  # noqa: F401
from .hierarchy import (SAParams, build_hierarchy, generate_problem, load_problem, permute_problem,  # noqa: F401
                        rcm_problem, split_problem)

__all__ = ["SequentialBackend", "DistributedBackend", "SAParams", "build_hierarchy",
           "generate_problem", "load_problem", "permute_problem", "rcm_problem", "split_problem", "save_hierarchy",
           "load_hierarchy"]
