mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_parity_gpu.py -v --timeout 150 --timeout-method thread -m gpu -k "softdot or shift or group_barrier or persistent_barrier or policy_head or two_streams or aliased or train_parity" > gpurun_out/t4.log 2>&1
rc=$?; echo tests_rc=$rc; grep -E "PASS|FAIL|Error" gpurun_out/t4.log | head -40
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 200 python -m dasa_amd.kbench 20 > gpurun_out/kb20.json 2>gpurun_out/kb20.err; echo kb_rc=$?
timeout -k 10 300 python tools/x6_shapes.py --forms 8,10,11,7,12,13 > gpurun_out/x6_prio.txt 2>&1; echo x6_rc=$?
cat gpurun_out/x6_prio.txt
