set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/churn
for k in routes deliveries match; do
  timeout -k 10 300 python -u tools/bench_churn.py --kind $k > gpurun_out/churn/$k.json 2> gpurun_out/churn/$k.log || exit 1
done
timeout -k 10 300 python -u tools/bench_acl.py > gpurun_out/churn/acl.json 2> gpurun_out/churn/acl.log || exit 1
