# Round-4 call 3: GPU parity suite + smoke on the new CRC default, then one
# bench line per configs[1]-[4] mode with its same-run CPU baseline and the
# full oracle check of every block (scripts/gpu_r4_suite.sh lines1).
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r3_tests.sh r4c && bash scripts/gpu_r4_suite.sh r4c lines1
