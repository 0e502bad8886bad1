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

# Test plumbing only: pageable torch copies of more than ~1 MiB (fixtures to
# the device, results back) would make the HIP runtime page-lock the numpy
# buffer and DMA it on an SDMA engine; below its pinned-transfer minimum it
# copies through its own pinned staging buffer instead.  The three rare
# illegal addresses on record were all raised by such a copy right after a
# clean synchronize (profiles/r05/pageable_path/), so the
# suite keeps its own copies on the staging path.  The library never hands
# the runtime a pageable buffer for a DMA (kvh.hip: is_pinned -> bounce), and
# the register -> DMA -> unregister -> free tests still run as before.  Set
# GPU_PINNED_MIN_XFER_SIZE yourself (MiB; on the box 1 MiB copies still
# staged and 2.4 MB ones were locked) to restore the runtime's default path.  Must precede HIP initialisation.
os.environ.setdefault("GPU_PINNED_MIN_XFER_SIZE", "1024")
