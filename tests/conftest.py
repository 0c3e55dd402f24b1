import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

SCENES = os.path.join(ROOT, "tests", "golden", "scenes")
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
