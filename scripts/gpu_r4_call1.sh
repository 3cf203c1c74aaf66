# Round-4 first call: GPU parity suite + smoke on a fresh box, then the SQ
# (LDS / VALU busy) passes and the first half of the FETCH / WRITE passes of
# the measurement suite (scripts/gpu_r3_suite.sh), for scripts/pmc_r3.py.
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r3_tests.sh r4a pmc2 && bash scripts/gpu_r3_suite.sh r4a pmc1a
