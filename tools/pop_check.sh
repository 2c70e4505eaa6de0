set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/pop
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_fused_env.py -k "population or headline_rollout or rank_sizes or multi_tile" -x -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/pop/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pop/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --config pbt --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/pop/pbt$i.json 2> gpurun_out/pop/pbt$i.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/pop/pbt$i.json').read().strip().splitlines()[-1]); print('pbt', round(d['ms_per_step'],3))"
done
VARIANTS="base base" bash tools/variants_bench.sh
