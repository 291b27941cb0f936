cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; tail -2 gpurun_out/pytest_gpu.log
for cfg in c4 frank; do for L in flipcomplexityempirical_amd/libA.so flipcomplexityempirical_amd/libB.so; do
  v=$(FLIPWALK_LIB=$L timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline --steps 5 | python -c "import json,sys; print('%.4e' % json.loads(sys.stdin.read().strip().splitlines()[-1])['value'])")
  echo "$cfg $(basename $L) $v"; done; done
