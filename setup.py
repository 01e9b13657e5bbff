"""setuptools hook: compile the native extensions in-tree before the package files are collected.

* ``symmetry_amd/_C.so``         -- gfx950 HIP kernels + RCCL wrapper (needs hipcc; skipped with a
  warning when ROCm is absent, which leaves a proxy-mode-only install);
* ``symmetry_amd/net/_native.so`` -- crypto / Noise / secretstream / epoll transport (g++ + OpenSSL).

The build itself lives in :mod:`symmetry_amd._build` (also ``python -m symmetry_amd._build``).
"""
import os
import shutil
import sys

from setuptools import find_packages, setup
from setuptools.command.build_py import build_py


class BuildNative(build_py):
    def run(self):
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from symmetry_amd import _build

        _build.build_net()
        if shutil.which("hipcc") or os.path.exists("/opt/rocm/bin/hipcc"):
            _build.build_kernels()
        else:
            print("warning: hipcc not found -- GPU kernels not built (proxy mode only)", file=sys.stderr)
        super().run()


setup(
    name="symmetry-amd",
    version="1.0.0",
    description="MI355X-native peer-to-peer LLM inference provider (symmetry-cli): CDNA4 HIP kernels + RCCL",
    long_description=open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "README.md")).read(),
    long_description_content_type="text/markdown",
    python_requires=">=3.10",
    license="MIT",
    packages=find_packages(include=["symmetry_amd", "symmetry_amd.*"]),
    package_data={"symmetry_amd": ["_C.so", "net/_native.so"]},
    install_requires=["torch>=2.4", "numpy", "pyyaml", "aiohttp"],
    extras_require={"hf": ["safetensors", "tokenizers"], "test": ["pytest", "pytest-timeout", "hypothesis"]},
    entry_points={
        "console_scripts": [
            "symmetry-cli = symmetry_amd.cli:main",            # the provider (reference: src/symmetry.ts)
            "symmetry-dht = symmetry_amd.net.discovery:main",  # discovery / bootstrap node (DHT analogue)
            "symmetry-server = symmetry_amd.cli:server_main",  # local Symmetry server
            "symmetry-client = symmetry_amd.cli:client_main",  # minimal streaming client
        ]
    },
    cmdclass={"build_py": BuildNative},
)
