import importlib.util
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


def load_pkg():
    """Import the host package from its hyphenated directory (aiyagari-replication_amd/)."""
    name = "aiyagari_replication_amd"
    if name in sys.modules:
        return sys.modules[name]
    root = ROOT / "aiyagari-replication_amd"
    spec = importlib.util.spec_from_file_location(name, root / "__init__.py",
                                                  submodule_search_locations=[str(root)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="session")
def pkg():
    return load_pkg()


@pytest.fixture(scope="session")
def golden():
    def get(name):
        return dict(np.load(GOLDEN / f"{name}.npz", allow_pickle=False))
    return get


@pytest.fixture(scope="session")
def gpu(pkg):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    # the product path must be the HIP library: loading it here is part of the check
    pkg.lib()
    return torch.device("cuda:0")
