import glob
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def golden(name):
    """Load a committed fixture (npz, no pickles)."""
    with np.load(os.path.join(HERE, "golden", name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def golden_names(prefix):
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(HERE, "golden", prefix + "*.npz")))


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    den = np.linalg.norm(b.ravel())
    return np.linalg.norm((a - b).ravel()) / (den if den > 0 else 1.0)


@pytest.fixture(scope="session")
def oracle():
    import oracle_lib
    oracle_lib.lib()
    return oracle_lib


def load_kctc():
    """Import kaldi-ctc_amd/ (hyphenated dir) as the package `kaldi_ctc_amd`."""
    import importlib.util
    if "kaldi_ctc_amd" in sys.modules:
        return sys.modules["kaldi_ctc_amd"]
    pkg = os.path.join(ROOT, "kaldi-ctc_amd")
    spec = importlib.util.spec_from_file_location("kaldi_ctc_amd", os.path.join(pkg, "__init__.py"),
                                                  submodule_search_locations=[pkg])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["kaldi_ctc_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="session")
def kctc():
    return load_kctc()


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu-marked test run without a visible GPU")
    m = load_kctc()
    m.lib()  # fail loudly if the HIP library is missing
    return torch.device("cuda:0")
