set -euo pipefail
bash scripts/gpu_tests_dist.sh z3
bash scripts/gpu_bench_n2_gloo.sh
