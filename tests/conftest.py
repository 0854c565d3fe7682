import os
import sys

# fixed BLAS thread count: MKL's dynamic threading changes CPU float summation order under load,
# and the lr=0.5 oracle trajectories (test_oracle_golden) amplify that past their tolerance
os.environ.setdefault("MKL_DYNAMIC", "FALSE")
os.environ.setdefault("OMP_DYNAMIC", "FALSE")

import pytest  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long CPU test")


def golden_path(name):
    return os.path.join(GOLDEN, name)


@pytest.fixture(scope="session")
def golden():
    return golden_path


def bf16_close(got, ref, rtol=2e-2, atol_of_max=1e-2, norm_tol=1e-2):
    """The bf16 parity bar (north_star: 2e-2 for bf16), element by element and not only by norm:
    every element within rtol * |ref| + atol_of_max * max|ref| (the absolute part covers entries near
    zero, whose error is set by the bf16 rounding of the large terms that cancel there), the max error
    within rtol * max|ref|, and ||err|| / ||ref|| within norm_tol.  Returns (ok, stats) so a failing
    assert can show the numbers."""
    g = got.detach().double().cpu().flatten()
    r = ref.detach().double().cpu().flatten()
    e = (g - r).abs()
    rmax = float(r.abs().max()) + 1e-30
    worst = float((e / (rtol * r.abs() + atol_of_max * rmax)).max())
    stats = dict(worst_elem_ratio=worst, maxrel=float(e.max()) / rmax, normrel=float(e.norm() / (r.norm() + 1e-30)))
    return (worst <= 1.0 and stats["maxrel"] <= rtol and stats["normrel"] <= norm_tol), stats
