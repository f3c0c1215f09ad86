"""Build the netsdb_amd native extensions IN-TREE for gfx950 (MI355X).

    PYTORCH_ROCM_ARCH=gfx950 python setup.py build_ext --inplace

Two extensions:
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


def hip_ext():
    from torch.utils.cpp_extension import CUDAExtension

    srcs = [os.path.join(KDIR, f) for f in ("bindings.cpp", "gemm.hip", "conv2d.hip", "rowops.hip")]
    return CUDAExtension(
        name="netsdb_amd._hip_kernels",
        sources=srcs,
        include_dirs=[os.path.join(ROOT, KDIR)],
        extra_compile_args={
            "cxx": ["-O3", "-std=c++17"],
            "nvcc": ["-O3", "-std=c++17", "--offload-arch=gfx950", "-fno-gpu-rdc", "-munsafe-fp-atomics"],
        },
    )


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


def main():
    from torch.utils.cpp_extension import BuildExtension

    which = os.environ.get("NSDB_BUILD", "all")
    exts = []
    if which in ("all", "native"):
        exts.append(native_ext())
    if which in ("all", "hip"):
        exts.append(hip_ext())
    setup(
        name="netsdb_amd",
        version="0.1.0",
        packages=["netsdb_amd"],
        ext_modules=exts,
        cmdclass={"build_ext": BuildExtension.with_options(use_ninja=True)},
    )


if __name__ == "__main__":
    sys.exit(main())
