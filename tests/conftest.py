"""Shared pytest configuration.

Markers:
  gpu  — needs a real MI355X (run on the GPU box with `-m gpu`).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an AMD MI355X GPU (gfx950)")
    config.addinivalue_line("markers", "slow: long-running test")
