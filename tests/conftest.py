import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "llama.vk_amd"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(autouse=True)
def _gpu_heartbeat(request):
    """While a GPU test runs, append a line to gpurun_out/pytest_heartbeat.log every 20 s. The
    full-size parity tests run the reference CPU build for minutes (the 65B 512-token prompt
    at -t 16 takes ~3 min on a slow host) and print nothing meanwhile; the GPU-box runner
    takes a command that writes nothing to stdout, stderr or gpurun_out/ for 3 minutes to be
    hung and kills it."""
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    import threading
    import time
    d = os.path.join(ROOT, "gpurun_out")
    stop = threading.Event()

    def beat():
        t0 = time.time()
        while not stop.wait(20.0):
            try:
                os.makedirs(d, exist_ok=True)
                with open(os.path.join(d, "pytest_heartbeat.log"), "a") as f:
                    f.write("%s %.0f s\n" % (request.node.nodeid, time.time() - t0))
            except OSError:
                pass

    th = threading.Thread(target=beat, daemon=True)
    th.start()
    try:
        yield
    finally:
        stop.set()
        th.join(timeout=5)


def _ensure_built():
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "oracle"], stdout=subprocess.DEVNULL)
    if not os.path.exists(os.path.join(ROOT, "llama.vk_amd", "bin", "lvk-gen-model")):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "llama.vk_amd"),
                               os.path.join(ROOT, "llama.vk_amd", "bin", "lvk-gen-model")], stdout=subprocess.DEVNULL)


@pytest.fixture(scope="session")
def model_dir(tmp_path_factory):
    _ensure_built()
    return str(tmp_path_factory.mktemp("models"))


@pytest.fixture(scope="session")
def oracle():
    _ensure_built()
    from oracle_lib import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def ref():
    from oracle_lib import REF_SO, Ref
    if not os.path.exists(REF_SO):
        pytest.skip("reference build oracle/_ref/libref.so not present")
    return Ref()


TINY = {
    "tiny_q4_0": dict(n_embd=256, n_head=2, n_layer=32, ftype=2, seed=1),
    "tiny_q4_1": dict(n_embd=256, n_head=2, n_layer=40, ftype=3, seed=7),
    "tiny_l80_q4_0": dict(n_embd=256, n_head=2, n_layer=80, ftype=2, seed=3),
}


@pytest.fixture(scope="session")
def tiny_models(model_dir):
    from oracle_lib import gen_model
    return {k: gen_model(os.path.join(model_dir, k + ".bin"), **v) for k, v in TINY.items()}


@pytest.fixture(scope="session")
def gpu_available():
    import lvk
    if lvk.device_count() < 1:
        pytest.fail("no GPU visible to the gpu-marked test (HIP extension loaded, but no device)")
    return True


def pytest_sessionfinish(session, exitstatus):
    # one HIP runtime per process (lvk.py, profiles/r03_runtime_mix.md): a test that pulls
    # torch into the process that loaded the library fails the session
    if "lvk" in sys.modules and "torch" in sys.modules and os.environ.get("LVK_ALLOW_TORCH") != "1":
        sys.stderr.write("\nERROR: torch was imported into the test process that loaded libllama_vk_amd.so\n")
        session.exitstatus = 1
