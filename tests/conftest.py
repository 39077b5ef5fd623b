import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "query-engines_amd"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libqe_hip.so on cuda:0)")
    config.addinivalue_line("markers", "slow: full-size (BASELINE) configuration")


@pytest.fixture(scope="session")
def gpu_ctx():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test collected without a GPU (run with -m 'not gpu' on CPU hosts)")
    from kquery.columnar import Context

    return Context.get(0)
