"""In-tree build of the native library ``ipex_llm_amd/_C.so``.

Three kinds of translation units, compiled in parallel:
  * ``csrc/hip/*.hip``   gfx950 kernels       -> hipcc --offload-arch=gfx950
  * ``csrc/cpu/*.cpp``   host quantizers/GEMM -> g++ -O3 -fopenmp (no torch)
  * ``csrc/torch/*.cpp`` torch.library ops    -> hipcc (host C++, torch headers)
  * ``csrc/runtime/*.cpp`` serving runtime (scheduler / block manager, torch custom classes)
and linked into one shared object loaded with ``torch.ops.load_library``.
Objects are cached under ``build/obj`` and rebuilt when the source or any
header under ``csrc`` is newer.  Usage: ``python -m ipex_llm_amd._build``.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig
import time

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
# A/B builds: ILLM_BUILD_DEFS="-DFOO=1" ILLM_BUILD_TAG=foo -> build/obj_foo, _C_foo.so
# (loaded with IPEX_LLM_AMD_LIB=_C_foo.so).  ``--debug``: the device-check
# build (ILLM_DEVICE_DEBUG: launch-geometry / host-contract checks in the hot
# kernels, csrc/hip/illm_device.h ILLM_DCHECK_FAILS) -> _C_debug.so
if "--debug" in sys.argv and __name__ == "__main__":
    os.environ["ILLM_BUILD_DEFS"] = (os.environ.get("ILLM_BUILD_DEFS", "") + " -DILLM_DEVICE_DEBUG=1").strip()
    os.environ.setdefault("ILLM_BUILD_TAG", "debug")
_DEFS = os.environ.get("ILLM_BUILD_DEFS", "").split()
_TAG = os.environ.get("ILLM_BUILD_TAG", "")
OBJ = os.path.join(ROOT, "build", "obj" + (f"_{_TAG}" if _TAG else ""))
LIB = os.path.join(PKG, f"_C_{_TAG}.so" if _TAG else "_C.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")


def _torch_paths():
    import torch  # noqa: F401  (import only for the paths)
    tdir = os.path.dirname(torch.__file__)
    return (os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include"),
            os.path.join(tdir, "lib"))


def _headers_mtime() -> float:
    hs = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True) + \
        glob.glob(os.path.join(CSRC, "**", "*.cuh"), recursive=True)
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _deps_mtime(obj: str, fallback: float) -> float:
    """newest header this object was compiled against (its -MMD depfile);
    every header under csrc when there is no depfile yet"""
    try:
        with open(obj + ".d") as f:
            txt = f.read().replace("\\\n", " ")
    except OSError:
        return fallback
    deps = [d for d in txt.split(":", 1)[-1].split() if d.endswith((".h", ".cuh", ".hpp"))]
    try:
        return max((os.path.getmtime(d) for d in deps), default=0.0)
    except OSError:                      # a header was renamed or removed
        return fallback


def _cmd(src: str, obj: str):
    tinc, tapi, _ = _torch_paths()
    common = ["-O3", "-fPIC", "-std=c++17", "-I", CSRC, "-MMD", "-MF", obj + ".d", *_DEFS]
    if src.endswith(".hip"):
        extra = []
        if os.path.basename(src).startswith(("gemv_", "attn_prefill", "gemm_8p")):
            # keep the GEMV epilogue as scalar f32 FMAs: SLP-packed v_pk_fma_f32
            # beside MFMAs costs issue cycles on gfx950 (and blocks v_fma_mix)
            # and MFMA results in VGPRs (no v_accvgpr_read per 64-block readout)
            extra = ["-fno-slp-vectorize", "-mllvm", "-amdgpu-mfma-vgpr-form"]
            # not for gemv_int4_xm.hip (the decode XM forms, lowbit_gemv5.cuh
            # launch5_xm_int4s): with the VGPR form hipcc (ROCm 7.2) miscompiles
            # some of them (profiles/gemv5_xm_forms_r6.txt)
            if os.path.basename(src) == "gemv_int4_xm.hip":
                extra = ["-fno-slp-vectorize"]
        return [HIPCC, f"--offload-arch={ARCH}", "-Wno-pass-failed", *extra, *common, "-c", src, "-o", obj]
    if "/cpu/" in src:
        return ["g++", *common, "-fopenmp", "-march=x86-64-v3", "-c", src, "-o", obj]
    pyinc = sysconfig.get_paths()["include"]
    return [HIPCC, *common, "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-D_GLIBCXX_USE_CXX11_ABI=1",
            "-Wno-unused-result", "-Wno-deprecated-declarations",
            "-I", tinc, "-I", tapi, "-I", pyinc, "-c", src, "-o", obj]


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "hip", "*.hip")) +
                  glob.glob(os.path.join(CSRC, "cpu", "*.cpp")) +
                  glob.glob(os.path.join(CSRC, "torch", "*.cpp")) +
                  glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))


def build(verbose: bool = False, jobs: int | None = None, force: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    hdr = _headers_mtime()
    todo, objs = [], []
    for src in sources():
        rel = os.path.relpath(src, CSRC).replace(os.sep, "_")
        obj = os.path.join(OBJ, rel + ".o")
        objs.append(obj)
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(src), _deps_mtime(obj, hdr)):
            todo.append((src, obj))
    jobs = jobs or min(8, max(1, (os.cpu_count() or 4)))
    t0 = time.time()
    if todo:
        def run(so):
            src, obj = so
            cmd = _cmd(src, obj)
            t_start = time.time()
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
            # stamp the object with the compile START time: a source or header
            # edited while it compiled is then newer and rebuilds next time
            # (otherwise a stale object -- possibly with an older struct layout
            # than its neighbours -- would look up to date)
            os.utime(obj, (t_start, t_start))
            if verbose:
                print(f"[build] {os.path.relpath(src, ROOT)}", flush=True)
            return src
        with cf.ThreadPoolExecutor(jobs) as ex:
            list(ex.map(run, todo))
    need_link = todo or not os.path.exists(LIB) or any(os.path.getmtime(o) > os.path.getmtime(LIB) for o in objs)
    if need_link:
        _, _, tlib = _torch_paths()
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", LIB + ".tmp",
               f"-L{tlib}", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-lc10", "-lc10_hip", "-fopenmp",
               f"-Wl,-rpath,{tlib}"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(LIB + ".tmp", LIB)
    if verbose:
        print(f"[build] {LIB} ({len(todo)} objects rebuilt, {time.time() - t0:.1f}s)", flush=True)
    return LIB


if __name__ == "__main__":
    build(verbose=True, force="--force" in sys.argv)
