"""Build the in-tree HIP library ``libgpd.so`` (gfx950) with hipcc.

The library must live in-tree so that it travels to the GPU box with the repository snapshot.
"""
import os
import pathlib
import shutil
import subprocess

PKG_DIR = pathlib.Path(__file__).resolve().parent
CSRC = PKG_DIR / "csrc"
INCLUDE = PKG_DIR.parent / "include"
LIB_PATH = PKG_DIR / "libgpd.so"
SOURCES = [CSRC / "gpd.hip", CSRC / "gpd_kernels.h", CSRC / "gpd_device.h", CSRC / "gpd_ctrl.h", CSRC / "gpd_handoff.h", INCLUDE / "gpd.h"]
ARCH = os.environ.get("GPD_OFFLOAD_ARCH", "gfx950")


def hipcc():
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: cannot build the gfx950 HIP library")


def needs_build():
    if not LIB_PATH.exists():
        return True
    t = LIB_PATH.stat().st_mtime
    return any(src.stat().st_mtime > t for src in SOURCES)


def build(force=False, verbose=False, stamps=False, variant=None, defines=()):
    """Compile csrc/gpd.hip into libgpd.so for gfx950 (code object v5, loadable by the
    HIP runtime that ships inside the torch wheel).  stamps=True builds the diagnostic
    libgpd_stamps.so (phase timestamps, never loaded unless GPD_LIB points at it);
    variant="x" with -D `defines` builds libgpd_x.so for A/B experiments (scripts/ab_geom.sh)."""
    out = PKG_DIR / "libgpd_stamps.so" if stamps else LIB_PATH
    if variant:
        out = PKG_DIR / f"libgpd_{variant}.so"
    if not force and not stamps and not variant and not needs_build():
        return LIB_PATH
    tmp = out.with_suffix(".so.tmp")
    # kernarg preloading: the step kernel's leading scalar arguments arrive in SGPRs.
    # max-ilp scheduling: a step launch runs ONE wave per CU (thin blocks), so the default
    # occupancy-driven scheduler buys nothing and ILP within the wave is what hides latency.
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-mcode-object-version=5", "-O3", "-std=c++17",
           "-mllvm", "-amdgpu-kernarg-preload-count=12", "-mllvm", "-amdgpu-sched-strategy=max-ilp",
           "-fPIC", "-shared", "-Wall", "-Wno-unused-result", f"-I{INCLUDE}", "-o", str(tmp),
           str(CSRC / "gpd.hip")] + (["-DGPD_STAMPS"] if stamps else []) + [f"-D{d}" for d in defines]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError("hipcc failed:\n" + " ".join(cmd) + "\n" + res.stdout + res.stderr)
    if verbose and (res.stdout or res.stderr):
        print(res.stdout + res.stderr)
    os.replace(tmp, out)
    return out


POLICY_LIB = PKG_DIR / "libgpd_policy.so"
POLICY_SOURCES = [CSRC / "gpd_policy.hip", INCLUDE / "gpd_policy.h"]


def build_policy(force=False, verbose=False):
    """Compile csrc/gpd_policy.hip (the fused rollout policy, include/gpd_policy.h) into
    libgpd_policy.so for gfx950.  -ffp-contract=off: the parts written "as torch computes them"
    (Normal sample and log-density, the time-limit bootstrap, GAE) round every operation."""
    if not force and POLICY_LIB.exists() and all(src.stat().st_mtime <= POLICY_LIB.stat().st_mtime
                                                 for src in POLICY_SOURCES):
        return POLICY_LIB
    tmp = POLICY_LIB.with_suffix(".so.tmp")
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-mcode-object-version=5", "-O3", "-std=c++17", "-ffp-contract=off",
           "-fPIC", "-shared", "-Wall", f"-I{INCLUDE}", "-o", str(tmp), str(CSRC / "gpd_policy.hip")]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError("hipcc failed:\n" + " ".join(cmd) + "\n" + res.stdout + res.stderr)
    if verbose and (res.stdout or res.stderr):
        print(res.stdout + res.stderr)
    os.replace(tmp, POLICY_LIB)
    return POLICY_LIB


if __name__ == "__main__":
    print(build(force=True, verbose=True))
    print(build_policy(force=True, verbose=True))
