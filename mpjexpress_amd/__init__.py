"""mpjexpress_amd — MI355X-native (gfx950) reduction-collective path of MPJ Express.

The product is libmpjx.so (include/mpjx.h): hand-written HIP combine kernels plus RCCL/xGMI (or
in-process multicore) exchanges behind the reference's Intracomm/Op codes. This package is the thin
host mirror used by tests and bench.py; see DESIGN.md and INTEGRATION.md.
"""
from .mpi import (MPI, Datatype, Init, Intracomm, MPIException, Op, combine, run_multicore,  # noqa: F401
                  smp_world, unique_id)

__all__ = ["MPI", "Datatype", "Op", "Intracomm", "MPIException", "combine", "smp_world",
           "run_multicore", "unique_id", "Init"]
