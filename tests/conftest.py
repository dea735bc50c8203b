import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP extension")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from pyrecover_amd import _ext

    _ext.native()  # GPU tests must exercise the HIP path: fail loudly if it is missing
    return torch.device("cuda", 0)


@pytest.fixture
def attn_opts(cuda):
    """Setter for the attention kernel selection (pyrecover_amd._ext.set_attn_options); every
    option is restored to its default after the test."""
    from pyrecover_amd import _ext

    yield _ext.set_attn_options
    _ext.set_attn_options(fwd_pipe=None, fwd_thr=None, dkdv_impl=None, dq_pipe=None, dkdv_split=None, dkdv_kreg=None,
                          bwd_fused=None, bwd_window=None, fwd_order=None, dq_order=None, dkdv_order=None)
