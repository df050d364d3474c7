import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "cuda-raytracer_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
SCENES = ROOT / "tests" / "golden" / "scenes"
REFERENCE_MEDIA = Path("/root/reference/media/pathtracer")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libptcore.so HIP kernels)")
    lib = ROOT / "cuda-raytracer_amd" / "lib" / "libptcore.so"
    if not lib.exists():
        subprocess.run(["make", "-s", "-C", str(ROOT / "cuda-raytracer_amd"), "-j8"], check=True)
    if not (ROOT / "oracle" / "build" / "libptoracle.so").exists():
        subprocess.run(["make", "-s", "-C", str(ROOT / "oracle")], check=True)


def have_gpu():
    import ptrace
    return ptrace.device_count() > 0


@pytest.fixture(scope="session")
def gpu_ctx():
    if not have_gpu():
        pytest.skip("no GPU")
    import ptrace
    ctx = ptrace.Context(0)
    yield ctx
    ctx.close()


def load_fixture(name):
    import ptrace
    return ptrace.ArrayScene.load(SCENES / f"{name}.npz")
