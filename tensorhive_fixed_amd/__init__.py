"""tensorhive_fixed_amd -- an MI355X-native GPU reservation, monitoring and job-execution daemon
with the capabilities of TensorHive 1.1 (kivicode/TensorHive-Fixed), plus the gfx950 kernels and
RCCL data-parallel payload used to measure it.

Subpackages
-----------
models/    ORM entities (users, reservations, jobs, ...) and the Llama-3 payload model
ops/       hand-written HIP kernels for gfx950 (+ ctypes bindings, CPU references)
parallel/  process groups, flat-buffer DDP over RCCL/xGMI, topology-aware placement
utils/     dates, JWT, password hashing, logging helpers
"""
__version__ = "1.1.0+mi355x"
