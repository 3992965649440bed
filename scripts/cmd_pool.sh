# host-Bullet threshold A/B, then the Bullet path tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_snark.py -x -q -k "bullet_paths or large" --timeout 300 --timeout-method thread > gpurun_out/gpu_t.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_t.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_env.sh SPG_BULLET_HOST_MAX "16 32 64 128" 4
