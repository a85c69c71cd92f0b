"""kg_qdiv (the score quotient used by the NodeNUMAResource scorers, kg_common.h) equals int64
division on randomized and boundary operands (host build of the same header the kernels use)."""
import pathlib
import shutil
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_qdiv_matches_int64_division(tmp_path):
    exe = tmp_path / "qdiv_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", f"-I{ROOT / 'include'}",
                    f"-I{ROOT / 'koordinator_amd' / 'csrc'}", str(ROOT / "tests" / "native" / "qdiv_check.cpp"),
                    "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "3000000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "bad 0" in out.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_divmod64_fp_matches_int64_division(tmp_path):
    """The device path of kg_divmod64 (fp64 estimate + exact correction) on the host compiler."""
    exe = tmp_path / "divmod_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", f"-I{ROOT / 'include'}",
                    f"-I{ROOT / 'koordinator_amd' / 'csrc'}", str(ROOT / "tests" / "native" / "divmod_check.cpp"),
                    "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "1000000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "bad 0" in out.stdout
