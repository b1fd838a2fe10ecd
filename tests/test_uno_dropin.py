"""Drop-in tests: the reference Uno core (libuno built from /root/reference sources by
oracle/ref/Makefile) runs hs015 under the ipopt preset with our plugin selected by
linear_solver=HIPLDL (GPU) or ORACLE (CPU).  The GPU run must reproduce the golden trace exactly
(iterations, every factorization's inertia, factorization/solve counts) and the solution within
1e-10 relative (north_star)."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "oracle", "_ref", "uno_kkt_driver")
GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "hs015_uno_oracle.json")))

needs_driver = pytest.mark.skipif(not os.path.exists(DRIVER), reason="driver not built (needs /root/reference)")


def run(solver):
    out = subprocess.run([DRIVER, "hs015", f"linear_solver={solver}", "logger=SILENT"], capture_output=True,
                         text=True, timeout=120)
    line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
    return json.loads(line)


def test_golden_matches_survey_probe():
    """17 iterations, 24 factorizations, 18 solves, x, f of the in-container probe."""
    g = GOLDEN
    assert g["status"] == 0 and g["iterations"] == 17
    assert g["factorizations"] == 24 and g["solves"] == 18
    assert abs(g["primals"][0] - 0.500000009999) < 1e-11 and abs(g["primals"][1] - 1.99999994001) < 1e-10
    assert abs(g["objective"] - 306.499975495) < 1e-8


@needs_driver
def test_oracle_plugin_reproduces_golden():
    r = run("ORACLE")
    assert r["iterations"] == GOLDEN["iterations"]
    assert r["inertia_trace"] == GOLDEN["inertia_trace"]


@needs_driver
@pytest.mark.gpu
def test_hipldl_plugin_reproduces_golden():
    r = run("HIPLDL")
    assert r["status"] == GOLDEN["status"]
    assert r["iterations"] == GOLDEN["iterations"]
    assert r["factorizations"] == GOLDEN["factorizations"] and r["solves"] == GOLDEN["solves"]
    assert r["inertia_trace"] == GOLDEN["inertia_trace"]
    for a, b in zip(r["primals"], GOLDEN["primals"]):
        assert abs(a - b) <= 1e-10 * max(1.0, abs(b))
    assert abs(r["objective"] - GOLDEN["objective"]) <= 1e-10 * abs(GOLDEN["objective"])
