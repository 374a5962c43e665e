import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


try:  # let PyTorch initialise the HIP runtime before libketogpu.so touches it (device buffers in tests)
    import torch  # noqa: E402

    TORCH_GPU = torch.cuda.is_available()
except Exception:  # pragma: no cover
    TORCH_GPU = False


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running CPU test")
