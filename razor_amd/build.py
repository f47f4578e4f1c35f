"""Builds the native library librazor_fec.so (HIP kernels for gfx950 + C host
layer) in-tree, under razor_amd/lib/.

Two variants are produced; they differ only in the SIM_VIDEO_SIZE the drop-in
symbols flex_fec_generate/flex_fec_recover are compiled with (the batched
rfec_* API takes the payload capacity at run time):

    lib/librazor_fec.so        SIM_VIDEO_SIZE 1000 (the reference default, sim_proto.h:54)
    lib/librazor_fec_v1200.so  SIM_VIDEO_SIZE 1200 (the 1200-byte benchmark packets)

Usage: python -m razor_amd.build [--force]
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
LIBDIR = PKG / "lib"
OBJDIR = PKG / "lib" / "obj"
INCLUDE = ROOT / "include"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("RFEC_OFFLOAD_ARCH", "gfx950")

HIP_SRC = [CSRC / "rfec_kernels.hip", CSRC / "rfec_probe.hip", CSRC / "rfec_wire.hip", CSRC / "rfec_fill.hip",
           CSRC / "rfec_service.hip", CSRC / "rfec_hostio.hip"]
# built once per SIM_VIDEO_SIZE: the C host layer, by concern (rfec_host.c: errors, planner, batched device
# and wire API; rfec_dropin.c: drop-in symbols + resident service; rfec_hostmem.c: host-memory batches;
# rfec_sender.c: sender staging; rfec_rx.c: receiver ingestion and sessions), and the flex drop-in
HOST_SRC = ["rfec_host.c", "rfec_dropin.c", "rfec_hostmem.c", "rfec_sender.c", "rfec_rx.c"]
C_SRC = [CSRC / f for f in HOST_SRC] + [CSRC / "rfec_flex.c"]
NET_SRC = CSRC / "rfec_net.c"  # host-only (sockets), independent of SIM_VIDEO_SIZE
HEADERS = [INCLUDE / "razor_fec.h", INCLUDE / "razor_flex.h", CSRC / "rfec_internal.h", CSRC / "rfec_launch.h",
           CSRC / "rfec_host_internal.h"]

VARIANTS = {"librazor_fec.so": 1000, "librazor_fec_v1200.so": 1200}


def _hipcc() -> str:
    p = ROCM / "bin" / "hipcc"
    return str(p) if p.exists() else "hipcc"


def _stale(out: Path, deps) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"build step failed: {' '.join(map(str, cmd))}")
    return r


def build(force: bool = False, verbose: bool = False) -> dict:
    LIBDIR.mkdir(parents=True, exist_ok=True)
    OBJDIR.mkdir(parents=True, exist_ok=True)
    built = {}
    kobjs = []
    for src in HIP_SRC:
        kobj = OBJDIR / (src.stem + ".o")
        if force or _stale(kobj, [src] + HEADERS):
            _run([_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
                  f"-I{INCLUDE}", f"-I{CSRC}", "-c", str(src), "-o", str(kobj)])
            if verbose:
                print("built", kobj)
        kobjs.append(kobj)
    nobj = OBJDIR / "rfec_net.o"
    if force or _stale(nobj, [NET_SRC] + HEADERS):
        _run(["gcc", "-std=c99", "-O2", "-fPIC", "-Wall", "-Wextra", f"-I{INCLUDE}", f"-I{CSRC}",
              "-c", str(NET_SRC), "-o", str(nobj)])
    kobjs.append(nobj)
    for name, vsize in VARIANTS.items():
        hobjs = []
        for src in C_SRC:
            hobj = OBJDIR / f"{src.stem}_v{vsize}.o"
            if force or _stale(hobj, [src] + HEADERS):
                _run(["gcc", "-std=c99", "-O2", "-fPIC", "-Wall", "-Wextra", "-Wno-unused-parameter",
                      f"-DSIM_VIDEO_SIZE={vsize}", "-D__HIP_PLATFORM_AMD__", f"-I{ROCM / 'include'}",
                      f"-I{INCLUDE}", f"-I{CSRC}", "-c", str(src), "-o", str(hobj)])
            hobjs.append(hobj)
        so = LIBDIR / name
        if force or _stale(so, kobjs + hobjs):
            _run([_hipcc(), "-shared", "-fPIC", *map(str, kobjs), *map(str, hobjs), "-o", str(so),
                  f"-Wl,-soname,{name}", "-lpthread", "-lm"])
            if verbose:
                print("built", so)
        built[name] = so
    return built


HARNESS_SRC = ROOT / "tests" / "dropin" / "fec_test_harness.c"
HARNESS = LIBDIR / "fec_test_harness"
GROUP_BENCH_SRC = ROOT / "tools" / "dropin_group_bench.c"  # tools/: per-group drop-in cost (GPU box)
GROUP_BENCH = LIBDIR / "fec_dropin_group_bench"


def build_harness(force: bool = False, verbose: bool = False) -> Path:
    """tests/dropin/fec_test_harness.c (the reference's FEC tests replayed through
    the drop-in symbols, own code) linked to lib/librazor_fec.so, and
    tools/dropin_group_bench.c linked to lib/librazor_fec_v1200.so: test and
    measurement infrastructure, built next to the library so they travel with it."""
    for src, exe, lib, vsize in ((HARNESS_SRC, HARNESS, "librazor_fec.so", 1000),
                                 (GROUP_BENCH_SRC, GROUP_BENCH, "librazor_fec_v1200.so", 1200)):
        if force or _stale(exe, [src, LIBDIR / lib] + HEADERS):
            _run(["gcc", "-std=c99", "-O2", "-Wall", "-Wextra", f"-DSIM_VIDEO_SIZE={vsize}", f"-I{INCLUDE}", str(src),
                  "-o", str(exe), f"-L{LIBDIR}", f"-l:{lib}", "-Wl,-rpath,$ORIGIN"])
            if verbose:
                print("built", exe)
    return HARNESS


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    out = build(force="--force" in argv, verbose=True)
    out["fec_test_harness"] = build_harness(force="--force" in argv, verbose=True)
    for k, v in out.items():
        print(k, v)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
