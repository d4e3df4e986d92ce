"""In-tree builder for the scaling_amd native extensions (gfx950 HIP + C++ host code).

No hipify, no torch JIT: every ``csrc/**/*.hip`` is compiled by ``hipcc --offload-arch=gfx950`` and
``csrc/**/*.cpp`` by hipcc as host C++, then linked against torch's bundled HIP runtime into
``scaling_amd/_C<EXT_SUFFIX>``.  Objects are cached by content hash under ``build/``.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "objs"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
EXT_NAME = "_C"


def _torch_paths() -> tuple[list[str], list[str]]:
    import torch

    tdir = Path(torch.__file__).parent
    inc = [str(tdir / "include"), str(tdir / "include" / "torch" / "csrc" / "api" / "include"), "/opt/rocm/include"]
    lib = [str(tdir / "lib")]
    return inc, lib


def _hipcc() -> str:
    return os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _common_flags(inc: list[str]) -> list[str]:
    import torch

    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    flags = [
        "-O3",
        "-fPIC",
        "-std=c++17",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DUSE_ROCM=1",
        "-D__HIP_PLATFORM_AMD__=1",
        "-DTORCH_EXTENSION_NAME=" + EXT_NAME,
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        "-Wno-unused-result",
        "-Wno-deprecated-declarations",
        f"-I{CSRC}",
        f"-I{sysconfig.get_paths()['include']}",
    ]
    flags += [f"-I{p}" for p in inc]
    return flags


def _sources() -> list[Path]:
    """Sources of the torch/HIP extension ``_C`` (kernels + bindings)."""
    return sorted(list((CSRC / "kernels").glob("*.hip")) + [CSRC / "bindings.cpp", CSRC / "rehearsal.cpp", CSRC / "blaslt.cpp"])


def _data_sources() -> list[Path]:
    """Sources of the torch-free native data library ``_data``."""
    return sorted((CSRC / "data").glob("*.cpp"))


def _obj_for(src: Path, flags: list[str]) -> Path:
    h = hashlib.sha1()
    h.update(src.read_bytes())
    for hdr in sorted(CSRC.rglob("*.h")):
        h.update(hdr.read_bytes())
    h.update(" ".join(flags).encode())
    return BUILD / f"{src.stem}-{h.hexdigest()[:16]}.o"


def _check_kernel_stubs(so: Path) -> None:
    """Fail the build if a kernel launch references a host stub that was never emitted (seen with
    hipcc when a template kernel's body trips its host pass): such a library imports but cannot load."""
    r = subprocess.run(["nm", "-C", "--undefined-only", str(so)], capture_output=True, text=True)
    missing = [ln.strip() for ln in r.stdout.splitlines() if "__device_stub__" in ln]
    if missing:
        raise RuntimeError("kernel host stubs missing from the extension:\n" + "\n".join(missing))


# per-file device flags (source file name -> extra hipcc flags).  flash_fwd.hip without SLP vectorisation: hipcc
# otherwise packs pairs of the softmax's f32 adds / muls into v_pk_*_f32, which beside MFMAs cost more issue cycles
# than the two scalar instructions they replace (MI355X_MICROARCH.md, "price of one filler"); forward 879-887 ->
# 897-903 TF at the 7B shape, interleaved A/B, profiles/attn_slp_ab_r5.log.  The backward kernels measured neutral.
#
# The training-path kernels with fp32 arithmetic are all built without SLP vectorisation, for reproducibility: with the
# SLP-packed build (v_pk_mul_f32 / v_pk_fma_f32 with op_sel / neg modifiers) the inverse-RoPE pass of the attention
# backward returned a different last bit in 2-8 % of backwards whenever another process's waves shared the GPU (0 of
# 408 with the RoPE kernels unpacked, 16 of 408 packed in the same run; profiles/race_forensics_r6.md).  The
# decode-only GEMV / flash-decoding kernels keep SLP (their packed dot products are their speed).
_NO_SLP = ["-fno-slp-vectorize"]
_FILE_FLAGS: dict[str, list[str]] = {f: _NO_SLP for f in ("flash_fwd.hip", "flash_bwd.hip", "swiglu_rope.hip", "norm.hip",
                                                           "xent_embed_optim.hip", "elementwise.hip")}


def _env_file_flags() -> dict[str, list[str]]:
    """Build-variant A/B: ``SCALING_AMD_FILE_FLAGS="flash_fwd.hip,flash_bwd.hip:-fno-slp-vectorize;gemm.hip:-DX=1"``
    adds flags to the named sources (with ``SCALING_AMD_BUILD_OUT`` naming the variant's .so, loaded on the GPU box
    through ``SCALING_AMD_EXT_SO``, ``ops/_ext.py``)."""
    out: dict[str, list[str]] = {}
    for part in filter(None, os.environ.get("SCALING_AMD_FILE_FLAGS", "").split(";")):
        names, _, fl = part.partition(":")
        for n in names.split(","):
            out.setdefault(n.strip(), []).extend(fl.split())
    return out


def _compile(src: Path, flags: list[str]) -> Path:
    flags = flags + _FILE_FLAGS.get(src.name, []) + _env_file_flags().get(src.name, [])
    obj = _obj_for(src, flags)
    if obj.exists():
        return obj
    if src.suffix == ".hip":
        cmd = [_hipcc()] + flags + [f"--offload-arch={ARCH}", "-mcode-object-version=5", "-x", "hip"]
    else:
        # host-only TU (bindings, data-pipeline C++): plain g++, no device code generation
        cmd = [os.environ.get("CXX", "g++")] + flags + ["-fopenmp"]
    cmd += ["-c", str(src), "-o", str(obj) + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(str(obj) + ".tmp", obj)
    return obj


def ext_path() -> Path:
    out = os.environ.get("SCALING_AMD_BUILD_OUT")
    if out:
        return Path(out).resolve()
    return ROOT / "scaling_amd" / (EXT_NAME + sysconfig.get_config_var("EXT_SUFFIX"))


def data_ext_path() -> Path:
    return ROOT / "scaling_amd" / ("_data" + sysconfig.get_config_var("EXT_SUFFIX"))


def build_data(verbose: bool = True) -> Path:
    """Build the pure C++ data-pipeline module (pybind11, no torch/HIP dependency)."""
    import pybind11

    BUILD.mkdir(parents=True, exist_ok=True)
    srcs = _data_sources()
    flags = ["-O3", "-fPIC", "-std=c++17", f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]
    objs = []
    for src in srcs:
        obj = _obj_for(src, flags)
        if not obj.exists():
            cmd = [os.environ.get("CXX", "g++")] + flags + ["-c", str(src), "-o", str(obj) + ".tmp"]
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"compile failed: {src}\n{r.stderr}")
            os.replace(str(obj) + ".tmp", obj)
        objs.append(obj)
    out = data_ext_path()
    cmd = [os.environ.get("CXX", "g++"), "-shared", "-fPIC", "-o", str(out) + ".tmp"] + [str(o) for o in objs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed\n{r.stderr}")
    os.replace(str(out) + ".tmp", out)
    if verbose:
        print(f"[scaling_amd] built {out.name}", file=sys.stderr)
    return out


def build(verbose: bool = True, jobs: int | None = None) -> Path:
    inc, lib = _torch_paths()
    flags = _common_flags(inc)
    BUILD.mkdir(parents=True, exist_ok=True)
    srcs = _sources()
    jobs = jobs or min(8, os.cpu_count() or 4, len(srcs))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, flags), srcs))
    out = ext_path()
    h = hashlib.sha1("".join(str(o) for o in objs).encode()).hexdigest()[:16]
    stamp = BUILD / f"link-{h}.stamp"
    if out.exists() and stamp.exists():
        return out
    cmd = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(out) + ".tmp"] + [str(o) for o in objs]
    for p in lib:
        cmd += [f"-L{p}", f"-Wl,-rpath,{p}"]
    cmd += ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python", "-lamdhip64", "-lhipblaslt", "-lgomp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    _check_kernel_stubs(Path(str(out) + ".tmp"))
    os.replace(str(out) + ".tmp", out)
    for old in BUILD.glob("link-*.stamp"):
        old.unlink()
    stamp.touch()
    if verbose:
        print(f"[scaling_amd] built {out.name} from {len(srcs)} sources", file=sys.stderr)
    return out


def build_all(verbose: bool = True) -> None:
    build_data(verbose)
    build(verbose)


if __name__ == "__main__":
    build_all()
