mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q --timeout 150 --timeout-method thread -m gpu -k "softdot or shift or group_barrier or persistent_barrier" > gpurun_out/t5.log 2>&1
rc=$?; echo tests_rc=$rc; tail -3 gpurun_out/t5.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -m dasa_amd.kbench 20 256 > gpurun_out/kb.json 2>gpurun_out/kb.err; echo kb_rc=$?
python -c "
import json; d=json.load(open('gpurun_out/kb.json'))
for k in ['shift_attn','shift_attn_bwd','softdot','softdot_bwd','cand_logit','ada_gate','adain_musigma','step_chain','attn_modules','launch_floor','adain_attention_aggregate']: print(k, d[k]['B20'], d[k]['B256']['frac'])
"
