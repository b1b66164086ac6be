set -e
export SHD_LOCKSTEP=1
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fastpred.py tests/test_gpu_groupkeys.py tests/test_gpu_boundary.py tests/test_gpu_kat.py > gpurun_out/ls_tests.log 2>&1
echo tests-ok
timeout -k 10 300 python bench.py --config P3-dense > gpurun_out/ls_dense.json 2> gpurun_out/ls_dense.err
echo ls-dense; cat gpurun_out/ls_dense.json | cut -c1-400
SHD_BPOS=1 timeout -k 10 300 python bench.py --config P3-dense > gpurun_out/ls_dense_bpos.json 2> gpurun_out/ls_dense_bpos.err
echo ls-dense-bpos; cut -c1-400 gpurun_out/ls_dense_bpos.json
timeout -k 10 300 python bench.py --config P3 > gpurun_out/ls_p3.json 2> gpurun_out/ls_p3.err
echo ls-p3; cut -c1-400 gpurun_out/ls_p3.json
