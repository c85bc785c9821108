import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libfedagg on the device)")
    config.addinivalue_line("markers", "slow: large-size parity on the GPU box")


def pytest_terminal_summary(terminalreporter):
    """FEDN_AMD_POISON_REUSE=1 runs (fedn_amd/reuse.py): how many staging buffers were watched, how many
    freed blocks were handed back and poisoned, and how many were not handed back within the retry."""
    mod = sys.modules.get("fedn_amd.reuse")
    if mod is not None and mod.enabled():
        mod.drain()
        terminalreporter.write_line(f"poison-reuse knob: {mod.stats()}")
