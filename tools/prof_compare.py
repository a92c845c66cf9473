"""Aggregate a rocprofv3 --kernel-trace --stats CSV into bench.py's kernel families and print the
per-family average launch duration next to bench.py's HIP-event numbers (same command)."""
import csv
import json
import sys
from collections import defaultdict

FAMILY_PREFIX = [
    ("gemm_x6", ("gemm_f32x6_nt_kernel",)),
    ("gemm_x6_tn", ("gemm_f32x6_tn_kernel",)),
    ("gemm_bf16", ("gemm_bf16_nt_kernel",)),
    ("gemm_skinny", ("gemm_skinny_nt_kernel", "gemm_skinny_nn_kernel")),
    ("gemm", ("gemm_f32_kernel", "gemm_nt_k64_kernel", "gemm_nt_glds_kernel")),   # (split-K reduce apart)
    ("gemm_splitk_reduce", ("splitk_reduce_kernel",)),
    ("bilstm", ("bilstm_persist_fwd_kernel", "bilstm_step_fused_kernel", "bilstm_step_cell_kernel")),
    ("bilstm_bptt", ("bilstm_persist_bwd_kernel", "bilstm_bptt_step_kernel", "bilstm_bptt_cell_kernel")),
    ("mha", ("mha_fwd_kernel", "mha_bwd_kernel", "mha_bwd_lds_kernel")),
    ("layernorm", ("ln_fwd_kernel", "ln_bwd_kernel")),
    ("softdot/shift/cand", ("scores_kernel", "apply_fwd_kernel", "apply_bwd_kernel", "attn_fwd_kernel",
                            "attn_bwd_apply_kernel", "attn_bwd_scores_kernel", "attn_bwd_dp_kernel",
                            "attn_split_bwd_kernel", "attn_split_dots_kernel", "attn_split_ctx_kernel",
                            "attn_rows_fwd_kernel", "attn_dot_rows_kernel")),
    ("ada_gate", ("AdaFwdOp", "AdaBwdOp", "ada_gate_fwd_kernel", "ada_gate_bwd_kernel")),
    ("adain_musigma", ("adain_musigma",)),
    ("gather", ("gather_rows_kernel",)),
    ("lstm_cell", ("lstm_cell_fwd_kernel", "lstm_cell_bwd_kernel")),
    ("policy_head", ("policy_head_fwd_kernel", "policy_head_bwd_kernel")),
]


def family(name):
    base = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    for fam, pre in FAMILY_PREFIX:
        if any(p in base for p in pre):
            return fam
    return "other:" + base.replace("void ", "").replace("(anonymous namespace)::", "")[:60]


def main(stats_csv, bench_json=None):
    fam = defaultdict(lambda: [0, 0.0])
    total = 0.0
    for r in csv.DictReader(open(stats_csv)):
        f = fam[family(r["Name"])]
        f[0] += int(r["Calls"])
        f[1] += float(r["TotalDurationNs"])
        total += float(r["TotalDurationNs"])
    bench = {}
    if bench_json:
        line = [ln for ln in open(bench_json).read().splitlines() if ln.startswith('{"metric"') or ln.startswith('{"profile_only"')][-1]
        bench = json.loads(line).get("kernels", {})
    print(f"{'family':<34}{'calls':>8}{'total ms':>11}{'share':>8}{'avg us':>10}{'bench avg us':>14}")
    for k, (n, ns) in sorted(fam.items(), key=lambda kv: -kv[1][1])[:25]:
        b = bench.get(k, {}).get("avg_launch_us", "")
        print(f"{k:<34}{n:>8}{ns / 1e6:>11.2f}{ns / total:>8.3f}{ns / n / 1e3:>10.2f}{b!s:>14}")


if __name__ == "__main__":
    main(*sys.argv[1:])
