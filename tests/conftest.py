"""pytest configuration: `gpu` marks tests that need an MI355X (run with -m gpu)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (gfx950); parity tests through the C-ABI")


# Every output the binding allocates is filled with 0xA5 bytes before its
# kernel runs (raikv_amd/binding.py: set_poison_outputs), so a parity test
# sees an element no kernel wrote instead of what the caching allocator left
# there.
os.environ.setdefault("KVH_POISON_OUTPUTS", "1")
