import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "distributed-faas_amd"), os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


# the suite mixes torch users (sharded groups, gloo ranks) with plain library
# users in one process: torch's HIP runtime must be the first one loaded
# (faasbal._lib.load)
try:
    import torch  # noqa: F401
except Exception:
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: larger CPU-side cases")
