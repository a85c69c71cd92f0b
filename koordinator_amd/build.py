"""In-tree build of the native pieces (no JIT, no site-packages install).

* ``koordinator_amd/lib/libkoordgpu.so`` — the engine: HIP kernels for gfx950 + host row
  builders, exporting the C-ABI declared in ``include/koord_gpu.h``.
* ``oracle/build/libkoordoracle.so`` — the CPU restatement used as the parity checker
  (test infrastructure; never loaded by the product path).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "koordinator_amd", "csrc")
LIB_DIR = os.path.join(ROOT, "koordinator_amd", "lib")
ENGINE_SO = os.path.join(LIB_DIR, "libkoordgpu.so")
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "build", "libkoordoracle.so")

ARCH = os.environ.get("KG_OFFLOAD_ARCH", "gfx950")


def _run(cmd: list[str]) -> None:
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def _newer(target: str, sources: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def engine_sources() -> list[str]:
    names = ["kg_engine.hip", "kg_host.cpp", "kg_cpuset.cpp", "kg_comm.cpp", "kg_common.h", "kg_host.h", "kg_comm.h"]
    return [os.path.join(CSRC, n) for n in names] + [os.path.join(ROOT, "include", "koord_gpu.h")]


def build_engine(force: bool = False) -> str:
    """Each object is rebuilt only when its own sources are newer (the device object takes minutes; the host
    objects seconds), then the library is linked."""
    os.makedirs(LIB_DIR, exist_ok=True)
    if not force and not _newer(ENGINE_SO, engine_sources()):
        return ENGINE_SO
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    obj_dir = os.path.join(LIB_DIR, "obj")
    os.makedirs(obj_dir, exist_ok=True)
    common = ["-O3", "-fPIC", "-std=c++17", "-ffp-contract=off", "-Wall", "-Wno-unused-function"]
    hdr = [os.path.join(ROOT, "include", "koord_gpu.h"), os.path.join(CSRC, "kg_common.h"), os.path.join(CSRC, "kg_host.h")]
    objs = []
    for src, extra in (("kg_host.cpp", []), ("kg_cpuset.cpp", []), ("kg_comm.cpp", [os.path.join(CSRC, "kg_comm.h")])):
        obj = os.path.join(obj_dir, src.rsplit(".", 1)[0] + ".o")
        if force or _newer(obj, [os.path.join(CSRC, src), *hdr, *extra]):
            _run(["g++", *common, "-c", os.path.join(CSRC, src), "-o", obj])
        objs.append(obj)
    dev_obj = os.path.join(obj_dir, "kg_engine.o")
    if force or _newer(dev_obj, [os.path.join(CSRC, "kg_engine.hip"), os.path.join(CSRC, "kg_comm.h"), *hdr]):
        _run([hipcc, *common, f"--offload-arch={ARCH}", "-c", os.path.join(CSRC, "kg_engine.hip"), "-o", dev_obj])
    tmp = ENGINE_SO + ".tmp"
    _run([hipcc, "-shared", f"--offload-arch={ARCH}", dev_obj, *objs, "-lrt", "-o", tmp])
    os.replace(tmp, ENGINE_SO)
    return ENGINE_SO


BOUNDS_SO = os.path.join(LIB_DIR, "libkoordgpu_bounds.so")


def build_variant(tag: str, defines: list) -> str:
    """A measurement build of the engine (lib/libkoordgpu_<tag>.so, the device object compiled with `defines`),
    loaded through KG_ENGINE_SO by tools; never by the product or the tests."""
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    obj_dir = os.path.join(LIB_DIR, "obj")
    common = ["-O3", "-fPIC", "-std=c++17", "-ffp-contract=off", "-Wall", "-Wno-unused-function"]
    dev_obj = os.path.join(obj_dir, f"kg_engine_{tag}.o")
    _run([hipcc, *common, *defines, f"--offload-arch={ARCH}", "-c", os.path.join(CSRC, "kg_engine.hip"), "-o", dev_obj])
    objs = [os.path.join(obj_dir, n) for n in ("kg_host.o", "kg_cpuset.o", "kg_comm.o")]
    so = os.path.join(LIB_DIR, f"libkoordgpu_{tag}.so")
    _run([hipcc, "-shared", f"--offload-arch={ARCH}", dev_obj, *objs, "-lrt", "-o", so + ".tmp"])
    os.replace(so + ".tmp", so)
    return so


def build_bounds(force: bool = False) -> str:
    """The bounds-checked engine (-DKG_BOUNDS_CHECK): every index into the pipelined placement's shared buffers is
    checked on the device and a violation is reported by the next kg_place / kg_eval instead of faulting.  A debug
    library beside the product one (loaded through KG_ENGINE_SO by tests/test_bounds_gpu.py); not built by default."""
    if not force and not _newer(BOUNDS_SO, engine_sources()):
        return BOUNDS_SO
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    obj_dir = os.path.join(LIB_DIR, "obj")
    common = ["-O3", "-fPIC", "-std=c++17", "-ffp-contract=off", "-Wall", "-Wno-unused-function"]
    dev_obj = os.path.join(obj_dir, "kg_engine_bounds.o")
    _run([hipcc, *common, "-DKG_BOUNDS_CHECK", f"--offload-arch={ARCH}", "-c", os.path.join(CSRC, "kg_engine.hip"),
          "-o", dev_obj])
    objs = [os.path.join(obj_dir, n) for n in ("kg_host.o", "kg_cpuset.o", "kg_comm.o")]
    if not all(os.path.exists(o) for o in objs):
        raise RuntimeError("build the product engine first (its host objects are linked into the bounds build)")
    tmp = BOUNDS_SO + ".tmp"
    _run([hipcc, "-shared", f"--offload-arch={ARCH}", dev_obj, *objs, "-lrt", "-o", tmp])
    os.replace(tmp, BOUNDS_SO)
    return BOUNDS_SO


def oracle_sources() -> list[str]:
    return [os.path.join(ORACLE_DIR, "koord_oracle.c"), os.path.join(ORACLE_DIR, "cpu_accumulator.c")]


def build_oracle(force: bool = False) -> str:
    srcs = oracle_sources()
    os.makedirs(os.path.dirname(ORACLE_SO), exist_ok=True)
    if not force and not _newer(ORACLE_SO, [*srcs, os.path.join(ROOT, "include", "koord_gpu.h")]):
        return ORACLE_SO
    tmp = ORACLE_SO + ".tmp"
    _run(["gcc", "-O2", "-fPIC", "-shared", "-std=c11", "-ffp-contract=off", "-Wall", *srcs, "-o", tmp, "-lm", "-lpthread"])
    os.replace(tmp, ORACLE_SO)
    return ORACLE_SO


# AddressSanitizer + UndefinedBehaviorSanitizer builds of the host code (kg_host.cpp: row builders,
# config validation, the per-pair row evaluation shared with the kernels) and of the oracle, for the CPU
# test suite (tests/test_sanitizers_cpu.py).  Host code only: GPU sanitizers are not available.
SAN_DIR = os.path.join(ROOT, "build", "sanitize")
SAN_HOST_SO = os.path.join(SAN_DIR, "libkoordhost_asan.so")
SAN_ORACLE_SO = os.path.join(SAN_DIR, "libkoordoracle_asan.so")
SAN_FLAGS = ["-O1", "-g", "-fPIC", "-shared", "-ffp-contract=off", "-fno-omit-frame-pointer",
             "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"]


def build_sanitized(force: bool = False) -> tuple[str, str]:
    os.makedirs(SAN_DIR, exist_ok=True)
    inc = ["-I", os.path.join(ROOT, "include")]
    host_src = [os.path.join(CSRC, "kg_host.cpp"), os.path.join(CSRC, "kg_cpuset.cpp")]
    if force or _newer(SAN_HOST_SO, engine_sources()):
        _run(["g++", "-std=c++17", *SAN_FLAGS, *inc, *host_src, "-o", SAN_HOST_SO + ".tmp"])
        os.replace(SAN_HOST_SO + ".tmp", SAN_HOST_SO)
    srcs = oracle_sources()
    if force or _newer(SAN_ORACLE_SO, [*srcs, os.path.join(ROOT, "include", "koord_gpu.h")]):
        _run(["gcc", "-std=c11", *SAN_FLAGS, *inc, *srcs, "-o", SAN_ORACLE_SO + ".tmp", "-lm", "-lpthread"])
        os.replace(SAN_ORACLE_SO + ".tmp", SAN_ORACLE_SO)
    return SAN_HOST_SO, SAN_ORACLE_SO


def build_all(force: bool = False) -> None:
    build_oracle(force)
    build_engine(force)


if __name__ == "__main__":
    if "--variant" in sys.argv:   # python koordinator_amd/build.py --variant <tag> -DX=1 ...
        i = sys.argv.index("--variant")
        build_variant(sys.argv[i + 1], sys.argv[i + 2:])
    elif "--bounds" in sys.argv:
        build_bounds(force="--force" in sys.argv)
    else:
        build_all(force="--force" in sys.argv)
