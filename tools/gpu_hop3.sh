# hop-kernel: the engine / timeline GPU tests, then the section anatomy (diagnostics build)
set -o pipefail
tag=${1:-hq}
d=gpurun_out/${RLO_OUT:-r6}
mkdir -p $d
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_timeline.py tests/test_gpu_sharded.py -m gpu -x -v --timeout 120 --timeout-method thread > $d/tests_$tag.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $d/tests_$tag.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -u tools/hop_anatomy.py 8 > $d/anat_$tag.txt 2>&1 || exit $?
cat $d/anat_$tag.txt
