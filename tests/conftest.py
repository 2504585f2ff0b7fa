"""pytest configuration: the `gpu` marker, import paths, in-tree builds.

CPU tests (`-m "not gpu"`) cover the oracle against the golden vectors, host
logic, and that the C-ABI library loads and exports every declared symbol.
GPU tests (`-m gpu`) are the parity tests proper and call through the C-ABI.
"""
import os
import subprocess
import sys

# torch first: it brings its own libamdhip64 (SONAME libamdhip64.so.7); our
# library's DT_NEEDED on that SONAME then binds to the SAME runtime, so torch
# device pointers and streams are valid in libyouth_icp.so.
import torch  # noqa: F401  (plumbing: device memory for the device-API tests)
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "slam-rgbd_amd")
ORACLE = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, ORACLE, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def _ensure_built():
    need = [os.path.join(PKG, "libyouth_icp.so"), os.path.join(PKG, "libyouth_synth.so"),
            os.path.join(PKG, "slam_host_demo"), os.path.join(PKG, "batch_multi_demo"), os.path.join(PKG, "batch_rccl_demo"),
            os.path.join(PKG, "libyouth_dist.so")]
    if not all(os.path.exists(p) for p in need):
        subprocess.run(["make", "-C", PKG, "-j8"], check=True, stdout=subprocess.DEVNULL)
    if not os.path.exists(os.path.join(ORACLE, "liboracle.so")):
        subprocess.run(["make", "-C", ORACLE], check=True, stdout=subprocess.DEVNULL)


_ensure_built()


def oracle_like(ctx_or_lanes):
    """Context manager: the oracle's spec a9 reduction set to what a GPU
    align ran.  Pass an IcpContext after its align (its reduction mode and
    youth_icp_get_lanes partition), a lanes tuple (LANE32 with that
    partition), or None (EXACT).  Inside it, oracle.reduce / align /
    align_batch restate the GPU's sums lane for lane (fp32 lane sums, fp64
    finalize), so correspondence counts compare exactly and sums to fp64
    summation order."""
    import oracle
    import youth_icp
    lanes = ctx_or_lanes
    if isinstance(ctx_or_lanes, youth_icp.IcpContext):
        lanes = ctx_or_lanes.lanes() if ctx_or_lanes.reduction == youth_icp.REDUCE_LANE32 else None
    if lanes is None:
        return oracle.reduction("exact")
    return oracle.reduction("lane32", lanes)


def lanes_of(ctx):
    """The context's last-align partition, or None when it ran EXACT."""
    import youth_icp
    return ctx.lanes() if ctx.reduction == youth_icp.REDUCE_LANE32 else None


@pytest.fixture(scope="session")
def has_gpu():
    import youth_icp
    return youth_icp.device_count() > 0


@pytest.fixture(autouse=True)
def _gpu_guard(request, has_gpu):
    if request.node.get_closest_marker("gpu") and not has_gpu:
        pytest.fail("GPU test selected but no HIP device is visible")
