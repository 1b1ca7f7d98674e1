import importlib.util
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

MODEL_DIR = os.environ.get("NW_MODEL_DIR", "/tmp/nw_models")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


def load_whisper_rs():
    path = os.path.join(ROOT, "nobs-whisper_amd", "whisper_rs.py")
    spec = importlib.util.spec_from_file_location("whisper_rs", path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules["whisper_rs"] = mod
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="session")
def wrs():
    return load_whisper_rs()


def model_path(shape: str, seed: int = 0) -> str:
    from make_model import write_model
    os.makedirs(MODEL_DIR, exist_ok=True)
    p = os.path.join(MODEL_DIR, f"{shape}_s{seed}.bin")
    if not os.path.exists(p):
        write_model(p, shape, seed)
    return p


@pytest.fixture(scope="session")
def micro_model():
    return model_path("micro")


@pytest.fixture(scope="session")
def tiny_model():
    return model_path("tiny")


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        return json.load(f)


@pytest.fixture(autouse=True)
def _no_pdec_give_ups(request):
    """Every GPU test but the give-up test itself: no persistent decode launch gave up (a give-up re-runs
    the step on the per-kernel path, so results stay right while the step silently costs the 50 ms wait:
    VERDICT r4 weak 11)."""
    if request.node.get_closest_marker("gpu") is None or "give_up" in request.node.name:
        yield
        return
    L = request.getfixturevalue("wrs").lib()
    before = L.whisper_mi355x_pdec_give_ups(None)
    yield
    after = L.whisper_mi355x_pdec_give_ups(None)
    assert after == before, f"{after - before} persistent decode launch(es) gave up during {request.node.name}"
