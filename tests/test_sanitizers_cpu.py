"""the host C-ABI code (kg_host.cpp with the kernels' shared per-pair code of kg_common.h:
row builders, config validation, kg_row_eval / kg_row_commit / kg_row_eval_rsv) and the oracle, built
with -fsanitize=address,undefined (build.build_sanitized) and run over the edge-case workload of
tests/sanitize_workload.py in a child process with the ASan runtime preloaded.  GPU sanitizers are not
available on this pool, so the kernels themselves are covered by the parity tests only."""
import os
import subprocess
import sys

import pytest

from koordinator_amd import build

HERE = os.path.dirname(os.path.abspath(__file__))


def _asan_runtime():
    r = subprocess.run(["g++", "-print-file-name=libasan.so"], capture_output=True, text=True)
    path = r.stdout.strip()
    return path if os.path.isabs(path) and os.path.exists(path) else None


def test_host_code_and_oracle_under_asan_ubsan():
    rt = _asan_runtime()
    if rt is None:
        pytest.skip("libasan not available")
    host, orc = build.build_sanitized()
    pre = os.environ.get("LD_PRELOAD", "")
    env = dict(os.environ, LD_PRELOAD=(rt + (" " + pre if pre else "")),
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               KG_SANITIZED_HOST_SO=host, KGO_SANITIZED_SO=orc)
    r = subprocess.run([sys.executable, os.path.join(HERE, "sanitize_workload.py")], env=env, capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-6000:]
    assert "runtime error" not in r.stderr, r.stderr[-6000:]
    assert "ERROR: AddressSanitizer" not in r.stderr, r.stderr[-6000:]
    assert "sanitize workload ok" in r.stdout
