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

# Debug runs only: with KVH_LIB=tools/libkvh_checked.so
# (`make checked`, device-side bounds checks on the exact-order sort and the
# ingest kernels) and KVH_ASSERT_CHECKS=1, every GPU test ends by asserting
# that no check failed.  The suite itself runs the product library and the
# HIP runtime's default copy paths (no GPU_PINNED_MIN_XFER_SIZE override).
import pytest  # noqa: E402


@pytest.fixture(autouse=True)
def _device_bounds_checks(request):
    yield
    if os.environ.get("KVH_ASSERT_CHECKS") != "1" or request.node.get_closest_marker("gpu") is None:
        return
    import ctypes
    import torch
    from raikv_amd import lib
    torch.cuda.synchronize()
    out = (ctypes.c_uint64 * 4)()
    rc = lib.kvh_debug_checks(out)
    assert rc == 1, f"KVH_ASSERT_CHECKS=1 needs the checked build (kvh_debug_checks -> {rc})"
    assert out[0] == 0, f"device bounds check failed: count {out[0]} site {out[1]} value {out[2]} limit {out[3]}"
