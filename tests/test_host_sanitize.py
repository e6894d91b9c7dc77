"""Host sanitizer run (reference CMakeLists.txt:50-52,79-90: LLAMA_SANITIZE_ADDRESS /
_UNDEFINED): the CPU tests that drive the host runtime on caller bytes --
the ggjt loader on truncated / corrupt / fuzzed files, the tokenizer, the quantize tool and
ggml_quantize, the ABI checks, the ggml arena and graph builder (graph_test in build-only mode)
-- run again in a child process against llama.vk_amd/lib/asan (make -C llama.vk_amd asan: the
runtime compiled with -fsanitize=address,undefined on the host side only), with clang's ASan
runtime preloaded.  Any ASan or UBSan report stops the child (halt_on_error) and fails this
test with the report.  No GPU: the device code is the product's and never runs here."""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN_LIB = os.path.join(ROOT, "llama.vk_amd", "lib", "asan", "libllama_vk_amd.so")
TESTS = ["tests/test_host_inputs.py", "tests/test_abi.py", "tests/test_ggml_quantize.py", "tests/test_ggml_graph.py"]


def _asan_runtime():
    c = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    return c[-1] if c else None


def test_host_runtime_under_asan_ubsan(tmp_path):
    rt = _asan_runtime()
    if not rt:
        pytest.skip("clang ASan runtime not found")
    if not os.path.exists(ASAN_LIB):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "llama.vk_amd"), "-j8", "asan"],
                              stdout=subprocess.DEVNULL)
    log = str(tmp_path / "san")
    env = dict(os.environ, LD_PRELOAD=rt, LVK_LIB=ASAN_LIB,
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:log_path=" + log,
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1:log_path=" + log)
    p = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "not gpu"] + TESTS,
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=1200)
    reports = "".join(open(f).read() for f in glob.glob(log + "*"))
    assert not reports, reports[:4000]
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
