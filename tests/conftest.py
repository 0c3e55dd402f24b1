import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

SCENES = os.path.join(ROOT, "tests", "golden", "scenes")

# No on-disk cache of specialised code objects unless a test sets one (tests/test_spec_program.py):
# compile times and cache provenance stay what each test expects.
os.environ.setdefault("RT_SPEC_CACHE_DIR", "")


def _deterministic_kernels():
    """Renderers made by tests start with RT_OPT_SPECIALIZE 0: the library's default compiles every
    uploaded scene's kernels in the background and swaps them in when ready, which would make the
    kernel a test pins (deferred, wavefront, generic megakernel) depend on compile timing.  The
    specialised paths, and the default itself, are tested explicitly (tests/test_gpu_spec*.py)."""
    import tinyraytracerinrust_amd as T
    T.Renderer.default_specialize = 0


_deterministic_kernels()
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def scene_text(name: str) -> str:
    with open(os.path.join(SCENES, name if name.endswith(".scene") else name + ".scene")) as f:
        return f.read()


@pytest.fixture(scope="session")
def worldmap():
    """Register worldmap.png with the oracle (decoded by PIL, independent of the product)."""
    from oracle import oracle as O
    return O.register_texture_file("worldmap.png", os.path.join(SCENES, "worldmap.png"))
