"""Writes tests/golden/kats.json: known-answer data transcribed from the reference's own tests and
traces (no reference source is copied, only the numbers):

  * mumps_5x5      -- unotest/functional_tests/MUMPSSolverTests.cpp:14-27 (solution [1..5]) and
                      :40-61 (inertia (3,2,0)); eigenvalues recorded at :86-101
  * mumps_singular -- MUMPSSolverTests.cpp:63-83 (hs015/byrd matrix, expected inertia (1,1,2),
                      matrix_is_singular() == true)
  * hs015_kkt0     -- first ipopt-preset KKT of examples/hs015 as assembled by Uno
                      (SURVEY.md 8(c) FACT 2: reg diag | Hessian | barrier Sigma | J^T), N=6, nnz=18,
                      expected inertia of the augmented system (n, m, 0) = (4, 2, 0)
                      (Subproblem.cpp:74)
  * hs015_lsq      -- least-squares multiplier system [I J^T; J 0] (Preprocessing.cpp:42-62),
                      N=6, nnz=10 (FACT 1), at the initial point x0 = (-2, 1) with slacks
Run: python tests/golden/make_golden.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))

kats = {
    "mumps_5x5": {
        "n": 5,
        "rows": [0, 0, 1, 1, 2, 2, 4], "cols": [0, 1, 2, 4, 2, 3, 4],
        "vals": [2.0, 3.0, 4.0, 6.0, 1.0, 5.0, 1.0],
        "rhs": [8.0, 45.0, 31.0, 15.0, 17.0],
        "solution": [1.0, 2.0, 3.0, 4.0, 5.0], "solution_tol": 1e-8,
        "inertia": [3, 2, 0],
        "eigenvalues": [-7.83039207, 8.94059148, -3.50815575, 1.7888887, 4.60906763],
        "source": "unotest/functional_tests/MUMPSSolverTests.cpp:14-61,86-101",
    },
    "mumps_singular": {
        "n": 4,
        "rows": [0, 0, 0, 1, 1, 2, 3], "cols": [0, 0, 1, 1, 1, 2, 3],
        "vals": [-0.0198, 0.625075, -0.277512, -0.624975, 0.625075, 0.0, 0.0],
        "inertia": [1, 1, 2], "singular": True,
        "source": "unotest/functional_tests/MUMPSSolverTests.cpp:63-83",
    },
    "hs015_kkt0": {
        "n": 6, "n_variables": 4, "n_constraints": 2,
        "rows": [0, 1, 2, 3, 4, 5, 0, 0, 1, 0, 2, 3, 0, 1, 2, 0, 1, 3],
        "cols": [0, 1, 2, 3, 4, 5, 0, 1, 1, 0, 2, 3, 4, 4, 4, 5, 5, 5],
        "vals": [0, 0, 0, 0, 0, 0, 4402.0, 1468.0, 2069.33, 0.4, 100.0, 100.0, 1.0, -2.0, -1.0, 1.0, 2.0, -1.0],
        "regularization_size": 6, "expected_inertia": [4, 2, 0],
        "source": "SURVEY.md 8(c) FACT 2 (reference libuno.a + probe plugin), Subproblem.cpp:57-74",
    },
    "hs015_lsq": {
        "n": 6,
        "rows": [0, 1, 2, 3, 0, 1, 2, 0, 1, 3], "cols": [0, 1, 2, 3, 4, 4, 4, 5, 5, 5],
        "vals": [1.0, 1.0, 1.0, 1.0, 1.0, -2.0, -1.0, 1.0, 2.0, -1.0],
        "inertia": [4, 2, 0],
        "source": "Preprocessing.cpp:42-62 pattern, SURVEY.md FACT 1 (N=6, nnz=10)",
    },
}

if __name__ == "__main__":
    with open(os.path.join(HERE, "kats.json"), "w") as f:
        json.dump(kats, f, indent=1)
    print("wrote", os.path.join(HERE, "kats.json"))
