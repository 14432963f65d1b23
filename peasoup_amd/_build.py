"""In-tree native build driver (CMake + Ninja, hipcc for gfx950).

Builds ``peasoup_amd/_C*.so`` (pybind11 extension) and the ``bin/peasoup``,
``bin/peasoup_coincidencer``, ``bin/peasoup_tools`` and ``bin/psoup_unit_tests``
executables from ``csrc/``.  The artefacts stay in the repository tree so they
travel with the source snapshot to a GPU box.

``python peasoup_amd/_build.py --sanitize address`` (or ``undefined`` /
``thread``) builds only the host unit tests under that sanitizer into
``build-<sanitizer>/`` -> ``bin/psoup_unit_tests_<sanitizer>``.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
BUILD_DIR = REPO / "build"


def _jobs() -> int:
    env = os.environ.get("MAX_JOBS") or os.environ.get("CMAKE_BUILD_PARALLEL_LEVEL")
    if env and env.isdigit():
        return max(1, min(16, int(env)))
    return max(1, min(16, os.cpu_count() or 4))


def build(verbose: bool = False, clean: bool = False, sanitize: str = "") -> None:
    """Configure (once) and build every native target for gfx950 (or, with
    ``sanitize``, only the host unit tests under that host sanitizer)."""
    build_dir = BUILD_DIR if not sanitize else REPO / f"build-{sanitize}"
    if clean and build_dir.exists():
        shutil.rmtree(build_dir)
    env = dict(os.environ)
    env.setdefault("CMAKE_PREFIX_PATH", "/opt/rocm")
    env.setdefault("PYTORCH_ROCM_ARCH", "gfx950")
    hip_compiler = "/opt/rocm/lib/llvm/bin/clang++"
    if not (build_dir / "build.ninja").exists():
        cmd = [
            "cmake", "-S", str(REPO), "-B", str(build_dir), "-G", "Ninja",
            f"-DCMAKE_HIP_COMPILER={hip_compiler}",
            "-DCMAKE_HIP_ARCHITECTURES=gfx950",
            "-DCMAKE_BUILD_TYPE=Release",
            f"-DPython3_EXECUTABLE={sys.executable}",
            f"-DPSOUP_SANITIZE={sanitize}",
        ]
        subprocess.run(cmd, check=True, env=env, stdout=None if verbose else subprocess.DEVNULL)
    cmd = ["cmake", "--build", str(build_dir), "-j", str(_jobs())]
    if sanitize:
        cmd += ["--target", "psoup_unit_tests"]
    res = subprocess.run(cmd, env=env, capture_output=not verbose, text=True)
    if res.returncode != 0:
        out = (res.stdout or "") + (res.stderr or "")
        raise RuntimeError("native build failed:\n" + out[-8000:])


if __name__ == "__main__":
    san = ""
    if "--sanitize" in sys.argv:
        san = sys.argv[sys.argv.index("--sanitize") + 1]
    build(verbose="-v" in sys.argv, clean="--clean" in sys.argv, sanitize=san)
