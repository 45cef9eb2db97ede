# (applies the stacked-batch patch first: git apply scripts/exp/r05v_stacked_batches.patch; reverted after this A/B)
# Round-5 stacked batches: GPU tests of the stacked path and the batch tests, then the bench's
# batch line (stacked, the in-flight path, the GPU_MAX_HW_QUEUES=4 child).
set -u
export TMPDIR=/tmp
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stacked.py tests/test_gpu_parity.py tests/test_gpu_batch_many.py -x -v --timeout 300 --timeout-method thread -k "stacked or batch or config5" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|PASS|FAIL|Error" $O/pytest.log | tail -25; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --stress-steps 0 --many-frames 0 --no-cpu-baseline --no-profile-pass > $O/bench.log 2>&1 || exit $?
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05v/bench.log").read().strip().splitlines()[-1])
print("headline", d["value"], d["parity"])
b = d["batch"]
print("batch", b["value"], b["parity"], b["note"])
print("inflight path", b["inflight_path"]["value"], b["inflight_path"]["parity"])
print("hwq4", b.get("hwq4"))
PY
# notConnectedMarkers floods: stacked against many-floods mode, 8 and 92 per call
timeout -k 10 300 python -u scripts/stack_probe.py 8 1024 0,1 > $O/stack_nc8.log 2>&1; rc=$?; grep -v amdgpu $O/stack_nc8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/stack_probe.py 92 1024 1,0 > $O/stack_nc92.log 2>&1; rc=$?; grep -v amdgpu $O/stack_nc92.log; exit $rc
