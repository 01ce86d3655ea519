"""Training payloads launched by the job-execution module (torchrun templates)."""
