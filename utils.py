"""Reference-compatible helpers (reference utils.py)."""
import torch

from pyrecover_amd.cli import PRECISION_STR_TO_DTYPE, get_args, init_logger, set_default_dtype  # noqa: F401
from pyrecover_amd.optim.lr import build_lr_scheduler  # noqa: F401
from pyrecover_amd.utils.flops import get_num_flop_per_token, get_num_params  # noqa: F401
import logging

logger = logging.getLogger()


@torch.no_grad()
def clip_grad_norm_(parameters, grad_max_norm):
    grads = [p.grad for p in parameters if p.grad is not None]
    total_norm = torch.nn.utils.get_total_norm(grads, error_if_nonfinite=True)
    torch.nn.utils.clip_grads_with_norm_(parameters, grad_max_norm, total_norm)
    return total_norm
