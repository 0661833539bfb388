"""Shared test setup.

* registers the ``gpu`` marker (MI355X-only tests, run with ``-m gpu``);
* puts the repo root (for ``oracle``) and ``npe-pfn_amd`` (for the ``npe_pfn``
  host package) on sys.path.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "npe-pfn_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm GPU); parity tests through the C-ABI")
    config.addinivalue_line("markers", "slow: longer CPU test")
