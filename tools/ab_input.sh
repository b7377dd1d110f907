cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_serving.py -q -m gpu -k uint8 --timeout 120 --timeout-method thread 2>&1 | tail -2 || exit 1
for i in uint8 fp32 uint8; do timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --input $i | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$i', d['ms_per_step'])" || exit 1; done
