"""Build the netsdb_amd native extensions IN-TREE for gfx950 (MI355X).

    PYTORCH_ROCM_ARCH=gfx950 python setup.py build_ext --inplace

Two extensions (both compiled directly with hipcc / the host C++ compiler — no source translation):
  * netsdb_amd._hip_kernels — CDNA4 HIP kernels (MFMA block GEMM, fused implicit-GEMM conv2d,
    row softmax, bias/act, LSTM cell, embedding bag) + PyTorch bindings.
  * netsdb_amd._native      — host C++ runtime (page pool / buffer manager, partitioned page
    files, TCAP parser, hash partitioner, slab allocator) bound with pybind11; no torch dependency.
"""
import os
import sys

os.environ.setdefault("PYTORCH_ROCM_ARCH", "gfx950")

from setuptools import setup  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
KDIR = os.path.join("netsdb_amd", "csrc", "kernels")
RDIR = os.path.join("netsdb_amd", "csrc", "runtime")


HIP_SOURCES = ("gemm.hip", "gemm_f32.hip", "conv2d.hip", "rowops.hip", "strings.hip", "dedup.hip", "relops.hip",
               "relops_bind.cpp", "pipeline.hip", "pipeline_bind.cpp")
PER_FILE_FLAGS = {}          # per-source extra hipcc flags
SDIR = os.path.join("netsdb_amd", "csrc", "study")
STUDY_SOURCES = ("gemm_study.hip",)


def study_ext():
    from setuptools import Extension

    srcs = [os.path.join(SDIR, f) for f in ("study_bindings.cpp",) + STUDY_SOURCES]
    return Extension(name="netsdb_amd._hip_study", sources=srcs)


def hip_ext():
    """The kernel extension is compiled by :class:`HipBuildExt` with hipcc directly (gfx950 code
    objects, no source translation step); ``sources`` only lists the files for dependency tracking."""
    from setuptools import Extension

    srcs = [os.path.join(KDIR, f) for f in ("bindings.cpp",) + HIP_SOURCES]
    return Extension(name="netsdb_amd._hip_kernels", sources=srcs)


def _torch_flags(study: bool = False):
    import sysconfig

    import torch
    from torch.utils.cpp_extension import include_paths, library_paths

    inc = [f"-I{p}" for p in include_paths()] + [f"-I{sysconfig.get_paths()['include']}", f"-I{os.path.join(ROOT, KDIR)}"]
    defs = ["-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DTORCH_API_INCLUDE_EXTENSION_H",
            "-DTORCH_EXTENSION_NAME=" + ("_hip_study" if study else "_hip_kernels"), f"-D_GLIBCXX_USE_CXX11_ABI={int(torch._C._GLIBCXX_USE_CXX11_ABI)}"]
    libdirs = library_paths()
    libs = [f"-L{d}" for d in libdirs] + [f"-Wl,-rpath,{d}" for d in libdirs] + [
        "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip", "-ltorch_hip"]
    return inc, defs, libs


def build_hip_extension(out_path: str, build_dir: str, jobs: int = 8, study: bool = False):
    """hipcc every kernel TU for gfx950 (parallel), the bindings TU as host C++, then link. ``study`` builds the
    separate diagnostic extension (_hip_study: the GEMM study variants) instead of the product one."""
    import subprocess
    from concurrent.futures import ThreadPoolExecutor

    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    hipcc = os.path.join(rocm, "bin", "hipcc")
    arch = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
    inc, defs, libs = _torch_flags(study)
    os.makedirs(build_dir, exist_ok=True)
    common = ["-O3", "-std=c++17", "-fPIC"] + defs + inc
    cmds, objs = [], []
    srcdir = SDIR if study else KDIR
    for f in (("study_bindings.cpp",) + STUDY_SOURCES) if study else (("bindings.cpp",) + HIP_SOURCES):
        src = os.path.join(ROOT, srcdir, f)
        obj = os.path.join(build_dir, f + ".o")
        objs.append(obj)
        hdrs = [os.path.join(ROOT, d, h) for d in (KDIR, srcdir) for h in os.listdir(os.path.join(ROOT, d))
                if h.endswith((".h", ".inc"))]
        if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(x) for x in [src] + hdrs):
            continue
        if f.endswith(".hip"):
            cmds.append([hipcc, "-x", "hip", f"--offload-arch={arch}", "-fno-gpu-rdc", "-munsafe-fp-atomics"]
                        + common + PER_FILE_FLAGS.get(f, []) + ["-c", src, "-o", obj])
        else:
            cmds.append([hipcc, "-x", "c++"] + common + [f"-I{rocm}/include", "-c", src, "-o", obj])

    def run(c):
        print(" ".join(c[:3] + [c[-3]]), flush=True)
        subprocess.run(c, check=True)

    with ThreadPoolExecutor(max(1, min(jobs, len(cmds) or 1))) as ex:
        list(ex.map(run, cmds))
    os.makedirs(os.path.dirname(out_path), exist_ok=True)
    subprocess.run([hipcc, "-shared", "-fPIC", f"--offload-arch={arch}", "-o", out_path] + objs + libs
                   + [f"-L{rocm}/lib", "-lamdhip64", "-lhiprtc"], check=True)


def native_ext():
    import pybind11
    from setuptools import Extension

    srcs = sorted(os.path.join(RDIR, f) for f in os.listdir(os.path.join(ROOT, RDIR)) if f.endswith(".cpp"))
    return Extension(
        "netsdb_amd._native",
        sources=srcs,
        include_dirs=[pybind11.get_include(), os.path.join(ROOT, RDIR)],
        extra_compile_args=["-O3", "-std=c++17", "-fvisibility=hidden", "-Wall", "-Wno-unused-function"],
        extra_link_args=["-lpthread"],
        language="c++",
    )


def _build_ext_cls():
    from setuptools.command.build_ext import build_ext

    class HipBuildExt(build_ext):
        def build_extension(self, ext):
            if ext.name in ("netsdb_amd._hip_kernels", "netsdb_amd._hip_study"):
                study = ext.name.endswith("_study")
                build_hip_extension(self.get_ext_fullpath(ext.name),
                                    os.path.join(self.build_temp, "hip_study" if study else "hip"),
                                    int(os.environ.get("MAX_JOBS", "8")), study=study)
            else:
                super().build_extension(ext)

    return HipBuildExt


def main():
    # the product build: the host runtime + the kernel extension. The GEMM study extension (_hip_study, the
    # diagnostic variants behind profiles/r2_gemm1_study .. r4_vendor) is opt-in: NSDB_BUILD=study
    which = os.environ.get("NSDB_BUILD", "all")
    exts = []
    if which in ("all", "native"):
        exts.append(native_ext())
    if which in ("all", "hip"):
        exts.append(hip_ext())
    if which == "study":
        exts.append(study_ext())
    setup(
        name="netsdb_amd",
        version="0.1.0",
        packages=["netsdb_amd"],
        ext_modules=exts,
        cmdclass={"build_ext": _build_ext_cls()},
    )


if __name__ == "__main__":
    sys.exit(main())
