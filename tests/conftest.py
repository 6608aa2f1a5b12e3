"""Shared pytest configuration.

`-m gpu` tests need a real MI355X and the in-tree HIP library; `-m "not gpu"`
tests run anywhere (oracle vs golden fixtures, host logic, C-ABI exports,
gloo multi-process tests).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built HIP library")
    config.addinivalue_line("markers", "slow: long-running")
