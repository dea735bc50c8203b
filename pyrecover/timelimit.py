from pyrecover_amd.timelimit import (  # noqa: F401
    TimeAwareStopper,
    get_job_end_time,
    get_remaining_time,
    monitor_timelimit,
)
