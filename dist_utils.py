"""Reference-compatible module path (reference dist_utils.py)."""
from pyrecover_amd.parallel.dist import (  # noqa: F401
    get_rank,
    get_slurm_job_end_time_env,
    is_distributed_activated,
    is_distributed_slurm_env,
    is_rank0,
    is_rank_eq,
    log_rank,
    log_rank0,
    maybe_cleanup_distributed,
    maybe_init_distributed,
)
