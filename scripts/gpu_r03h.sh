#!/bin/bash
# Round 3: parallel direct-DFT stage (odd prime lengths) + LDS twiddles for
# every per-wave length: stamp/app/parity tests, the star-stamp bench. Usage: TAG
set -o pipefail
TAG=${1:-r03h}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
PYT="python -u -m pytest -m gpu -v -s -rf -p no:cacheprovider --timeout 240 --timeout-method thread"
timeout -k 10 500 $PYT tests/test_gpu_stamps.py tests/test_gpu_app.py tests/test_gpu_parity.py tests/test_gpu_persist.py > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "FAILED|^E  |passed|failed|correctly rounded|parted" gpurun_out/${TAG}_tests.log | cut -c1-400 | tail -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python bench.py --config stamps31 --steps 3 --warmup 1 --no-cpu > gpurun_out/${TAG}_stamps.json 2> gpurun_out/${TAG}_stamps.err || { echo "stamps bench failed"; tail -5 gpurun_out/${TAG}_stamps.err; exit 3; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_stamps.json'));r=d['roofline'];print('stamps', round(d['value']), d['vs_baseline'], r['kernel'], r['frac'], [(k, round(v['ms_total'],1)) for k,v in r['kernels'].items()], [(k, round(v['ms_total'],1)) for k,v in r['phase_kernels']['kernels'].items()])"
