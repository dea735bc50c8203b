from pyrecover_amd.resubmit import ResubmitConfig, maybe_resubmit, resubmit_command, setup_resubmission  # noqa: F401
