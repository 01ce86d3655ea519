"""Data-parallel runtime over RCCL (backend "nccl" on ROCm) and xGMI-aware placement."""
