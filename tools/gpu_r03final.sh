# final-tree check (r03final: pipelined forward affine default): full GPU suite, smoke, default bench line
set -e
mkdir -p gpurun_out/r03final
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03final/gpu_tests.log 2>&1
echo "tests: $(tail -1 gpurun_out/r03final/gpu_tests.log)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03final/smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/r03final/bench.json 2> gpurun_out/r03final/bench.err
echo "bench done"
