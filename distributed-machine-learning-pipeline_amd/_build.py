"""In-tree build of the native extension ``hipdsml._C`` for gfx950.

No hipify, no JIT cache: every ``.hip`` kernel TU and every runtime ``.cpp`` is
compiled by ``hipcc --offload-arch=gfx950`` into ``<repo>/build/obj`` and
linked with the PyTorch binding TU into ``<package>/_C.so``, which travels to
the GPU box with the repository snapshot.  Objects are rebuilt when their
source or any header under ``csrc/`` is newer.

Usage:  python -m hipdsml._build [--force] [-j N] [--measure]

``--measure`` makes a measurement build (-DHIPDSML_MEASURE, objects under
``build/obj_measure``): the profiling knobs of csrc/kernels/common.h
``DSML_MEASURE_KNOB`` (traffic-dropping, grid-growing) become live and
``_C.measure_build`` is True.  Tools that need them build it, measure, and
run the default build again; every default build relinks the production
module (the flavor of the last link is recorded next to the objects), and the
GPU tests refuse to run on a measurement build.
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
REPO = PKG.parent
OBJ = REPO / "build" / "obj"
OUT = PKG / "_C.so"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")


def _torch_paths():
    import torch  # noqa: F401  (only for paths)
    from torch.utils import cpp_extension as ce

    try:
        inc = ce.include_paths(device_type="cuda")
        lib = ce.library_paths(device_type="cuda")
    except TypeError:  # older signature
        inc = ce.include_paths(True)
        lib = ce.library_paths(True)
    import torch as _t

    abi = int(_t._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _sources():
    kernels = sorted((CSRC / "kernels").glob("*.hip"))
    runtime = sorted((CSRC / "runtime").glob("*.cpp"))
    return kernels, runtime, CSRC / "bindings.cpp"


def _headers_mtime() -> float:
    hs = list(CSRC.rglob("*.h"))
    return max((h.stat().st_mtime for h in hs), default=0.0)


def _compile(src: Path, obj: Path, flags: list[str]) -> tuple[Path, str]:
    cmd = [HIPCC] + flags + ["-c", str(src), "-o", str(obj)]
    p = subprocess.run(cmd, capture_output=True, text=True)
    if p.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{p.stdout}\n{p.stderr}")
    return obj, p.stderr


def build(force: bool = False, jobs: int | None = None, verbose: bool = False,
          measure: bool = False) -> Path:
    kernels, runtime, binding = _sources()
    obj_dir = OBJ.parent / "obj_measure" if measure else OBJ
    obj_dir.mkdir(parents=True, exist_ok=True)
    flavor = "measure" if measure else "production"
    stamp = OBJ.parent / "linked_flavor"
    relink = not stamp.exists() or stamp.read_text().strip() != flavor
    inc, lib, abi = _torch_paths()
    extra = ["-DHIPDSML_MEASURE"] if measure else []
    base = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", str(CSRC),
            "-Wno-unused-result", "-Wno-pass-failed"] + extra
    host_only = ["-O3", "-std=c++17", "-fPIC", "-I", str(CSRC), "-D__HIP_PLATFORM_AMD__=1",
                 "-Wno-unused-result"] + extra
    torch_flags = host_only + [f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1",
                               "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
                               "-I", sysconfig.get_paths()["include"]]
    for p in inc:
        torch_flags += ["-I", p]
    hdr_t = _headers_mtime()
    jobs_todo = []
    objs = []
    for src in kernels:
        obj = obj_dir / (src.stem + ".hip.o")
        objs.append(obj)
        jobs_todo.append((src, obj, base))
    for src in runtime:
        obj = obj_dir / (src.stem + ".cpp.o")
        objs.append(obj)
        jobs_todo.append((src, obj, base))
    obj_b = obj_dir / "bindings.o"
    objs.append(obj_b)
    jobs_todo.append((binding, obj_b, torch_flags))

    stale = [(s, o, f) for (s, o, f) in jobs_todo
             if force or not o.exists() or o.stat().st_mtime < max(s.stat().st_mtime, hdr_t)]
    if stale:
        n = jobs or min(len(stale), int(os.environ.get("MAX_JOBS", "8")), os.cpu_count() or 4)
        with ThreadPoolExecutor(max_workers=max(1, n)) as ex:
            for obj, err in ex.map(lambda t: _compile(*t), stale):
                if verbose:
                    print(f"[hipdsml build] {obj.name}", file=sys.stderr)
                    if err.strip():
                        print(err, file=sys.stderr)
    newest = max(o.stat().st_mtime for o in objs)
    if force or stale or relink or not OUT.exists() or OUT.stat().st_mtime < newest:
        link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(OUT)]
        link += [str(o) for o in objs]
        for p in lib:
            link += ["-L", p, f"-Wl,-rpath,{p}"]
        link += ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
                 "-lamdhip64", "-lrccl", "-lrocprofiler-sdk-roctx"]
        p = subprocess.run(link, capture_output=True, text=True)
        if p.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(link)}\n{p.stdout}\n{p.stderr}")
        stamp.write_text(flavor)
    return OUT


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--measure", action="store_true",
                    help="measurement build (-DHIPDSML_MEASURE): profiling knobs live; tools only")
    a = ap.parse_args()
    out = build(force=a.force, jobs=a.j, verbose=True, measure=a.measure)
    print(out)


if __name__ == "__main__":
    main()
