#!/bin/bash
# Golden vectors of the IPM vector work (barrier diagonal Sigma, augmented right-hand side, primal-dual
# direction with the fraction-to-boundary step lengths) computed by the REFERENCE code: oracle/ref/ipm_fixtures
# links the Uno core compiled from /root/reference (oracle/ref/Makefile) and calls
# PrimalDualInteriorPointProblem::evaluate_lagrangian_hessian, Subproblem::assemble_augmented_rhs and
# Subproblem::assemble_primal_dual_direction on seeded inputs.  Run from the repository root.
set -euo pipefail
make -s -C oracle && make -s -j8 -C oracle/ref fixtures
oracle/_ref/ipm_fixtures > tests/golden/ipm_reference_vectors.json
# the reference's own augmented-matrix assembly (COOFormat::reset + Subproblem::
# assemble_augmented_matrix through the ipopt reformulation chain) for the arrowband model, with the inputs of
# the device assembly (uno_kkt_assemble_augmented); tests/test_ipm_vectors.py compares bit for bit
oracle/_ref/ipm_fixtures augmented > tests/golden/augmented_reference_vectors.json
