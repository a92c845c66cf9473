// Policy head of one decision step (agent_dg.py:832-886): candidate mask, teacher cross-entropy
// (CrossEntropyLoss(ignore_index=-100, reduction='sum'), agent_dg.py:251, 850), and the action:
// argmax with its log-probability, or a draw from Categorical(softmax(logit)) with its entropy and
// log-probability (agent_dg.py:862-880). The reference runs ~20 tiny PyTorch kernels here per step
// (masked_fill, log_softmax, nll, softmax, entropy, multinomial, log_prob, sums); this is one launch
// forward and one backward.
//
// One wave per batch row (C <= 256 candidates, up to 4 per lane), rows strided over the 16 waves of
// one workgroup; the CE row terms are summed in row order by wave 0 at the end (deterministic).
// Sampling is inverse-CDF on the counter RNG (dasa_uniform(seed, row)): the same distribution as
// torch.multinomial, another random stream.
// The sampled rollout's entropy and log-probability follow torch.distributions.Categorical(probs)
// exactly (agent_dg.py:874-880): its log-pmf is log(clamp(p, eps, 1 - eps)) with eps = FLT_EPSILON
// (probs_to_logits), so log_prob(a) and entropy = -sum p * log(clamp(p)) use the clamped logs and their
// gradients vanish where the clamp is active; argmax mode keeps the exact log_softmax
// (F.log_softmax(logit).gather, agent_dg.py:866-869).
#include "common.h"
#include "../../include/dasa_hip.h"

namespace {

constexpr int kVpl = 4;   // candidates per lane (C <= 256)
constexpr float kPEps = 1.1920928955078125e-07f;   // torch.finfo(float32).eps (clamp_probs)

__device__ __forceinline__ float clamped_log(float p) {   // log(clamp(p, eps, 1 - eps))
  return __logf(fminf(fmaxf(p, kPEps), 1.f - kPEps));
}

struct PolicyFwd {
  const float* logit; long ld;
  const int32_t* len;       // [B] valid candidates per row (mask = c >= len)
  const int64_t* target;    // [B] teacher action or ignore_index, or NULL (no CE)
  float* logp;              // [B][C] masked log-softmax (saved for backward; -inf where masked)
  float* ce_sum;            // [1] sum over rows of -logp[target] (rows with target == ignore skipped)
  float* ent;               // [B] entropy, or NULL
  float* logp_a;            // [B] log-probability of the chosen action, or NULL
  int64_t* action;          // [B] chosen action, or NULL (mode TEACHER); the input in mode FORCED
  float* ce_rows;           // [B] scratch
  int B, C, mode, ignore;
  uint64_t seed;
  const uint64_t* seed_src; // device seed source of a graph-captured launch (eff_seed), or null
};

__global__ __launch_bounds__(1024) void policy_head_fwd_kernel(PolicyFwd a) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int b = w; b < a.B; b += nw) {
    const int L = a.len[b];
    DASA_DCHECK(L >= 0 && L <= a.C, 16);
    DASA_DCHECK(!a.target || a.target[b] == a.ignore || (a.target[b] >= 0 && a.target[b] < a.C), 16);
    DASA_DCHECK(a.mode != DASA_POLICY_FORCED || (a.action[b] >= 0 && a.action[b] < L), 16);
    float z[kVpl];
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < kVpl; ++k) {
      const int c = lane + 64 * k;
      z[k] = (c < a.C && c < L) ? a.logit[(long)b * a.ld + c] : -INFINITY;
      m = fmaxf(m, z[k]);
    }
    m = wave_max(m);
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < kVpl; ++k) s += (z[k] == -INFINITY) ? 0.f : __expf(z[k] - m);
    s = wave_sum(s);
    const float lse = m + __logf(s);
    const bool cat = a.mode == DASA_POLICY_SAMPLE || a.mode == DASA_POLICY_FORCED ||
                     a.mode == DASA_POLICY_SAMPLE_ARGMAX;   // Categorical semantics
    float lp[kVpl], lc[kVpl], h = 0.f;
#pragma unroll
    for (int k = 0; k < kVpl; ++k) {
      const int c = lane + 64 * k;
      lp[k] = z[k] == -INFINITY ? -INFINITY : z[k] - lse;
      lc[k] = (cat && z[k] != -INFINITY) ? clamped_log(__expf(lp[k])) : lp[k];
      if (z[k] != -INFINITY) h -= __expf(lp[k]) * lc[k];
      if (c < a.C) a.logp[(long)b * a.C + c] = lp[k];
    }
    h = wave_sum(h);
    // teacher cross-entropy term
    float ce = 0.f;
    if (a.target) {
      const long t = a.target[b];
      if (t != a.ignore) {
        float v = -INFINITY;
#pragma unroll
        for (int k = 0; k < kVpl; ++k)
          if (lane + 64 * k == t) v = lp[k];
        v = wave_max(v);        // the one lane holding target t (-inf if t is masked: ce = +inf)
        ce = -v;
      }
    }
    // action
    int act = -1;
    if (a.mode == DASA_POLICY_ARGMAX || a.mode == DASA_POLICY_SAMPLE_ARGMAX) {   // first index of the max (torch.max)
      float best = -INFINITY;
      int bi = 0x7fffffff;
#pragma unroll
      for (int k = 0; k < kVpl; ++k) {   // ascending c: strict > keeps the first maximum
        const int c = lane + 64 * k;
        if (c < a.C && (z[k] > best || bi == 0x7fffffff)) { best = z[k]; bi = c; }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ob = __shfl_xor(best, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
      }
      act = bi;
    } else if (a.mode == DASA_POLICY_SAMPLE) {   // inverse CDF over the masked softmax
      const float u = dasa_uniform(eff_seed(a.seed, a.seed_src), (uint64_t)b);
      float carry = 0.f;
      int pick = 0x7fffffff, last = -1;
#pragma unroll
      for (int k = 0; k < kVpl; ++k) {
        const int c = lane + 64 * k;
        const float p = z[k] == -INFINITY ? 0.f : __expf(lp[k]);
        float incl = p;   // inclusive prefix sum over the lanes of this chunk
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const float y = __shfl_up(incl, o, 64);
          if (lane >= o) incl += y;
        }
        const float cum = carry + incl;
        if (p > 0.f && u < cum && c < pick) pick = c;
        if (p > 0.f) last = c;
        carry += __shfl(incl, 63, 64);
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        pick = min(pick, __shfl_xor(pick, o, 64));
        last = max(last, __shfl_xor(last, o, 64));
      }
      act = pick == 0x7fffffff ? last : pick;   // u beyond the rounded total: the last valid candidate
    } else if (a.mode == DASA_POLICY_FORCED) {   // the caller's action (it guarantees 0 <= action < len)
      act = (int)a.action[b];
    }
    if (lane == 0) {
      a.ce_rows[b] = ce;
      if (a.ent) a.ent[b] = h;
      if (a.action && act >= 0 && a.mode != DASA_POLICY_FORCED) a.action[b] = act;
    }
    if (a.logp_a && act >= 0) {
#pragma unroll
      for (int k = 0; k < kVpl; ++k)
        if (lane + 64 * k == act) a.logp_a[b] = lc[k];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {   // row-order sum: deterministic
    float t = 0.f;
    for (int b = 0; b < a.B; ++b) t += a.ce_rows[b];
    a.ce_sum[0] = t;
  }
}

struct PolicyBwd {
  const float* logp;        // [B][C] saved (exact log-softmax, -inf where masked)
  const int32_t* len;
  const int64_t* target;    // or NULL
  const int64_t* action;    // or NULL
  const float* ent;         // [B] saved entropy (unused: the row sums are recomputed)
  const float* d_ce;        // [1] or NULL
  const float* d_logp_a;    // [B] or NULL
  const float* d_ent;       // [B] or NULL
  float* dlogit; long ldd;
  int B, C, ignore, mode;
};

// One wave per row. With Categorical semantics (sample / forced): l_c = log(clamp(p_c)), u_c = 1 where
// the clamp is inactive; d log_prob(a) / dz_j = u_a (onehot_a - p_j); dH / dz_j = p_j (g_j - sum_c p_c g_c)
// with g_c = dH / dp_c = -(l_c + u_c). Argmax / teacher: u = 1 and l = log p (the exact log-softmax).
__global__ __launch_bounds__(1024) void policy_head_bwd_kernel(PolicyBwd a) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const bool cat = a.mode == DASA_POLICY_SAMPLE || a.mode == DASA_POLICY_FORCED || a.mode == DASA_POLICY_SAMPLE_ARGMAX;
  for (int b = blockIdx.x * nw + w; b < a.B; b += gridDim.x * nw) {
    const int L = a.len[b];
    float p[kVpl], gh[kVpl];
    float S = 0.f;
#pragma unroll
    for (int k = 0; k < kVpl; ++k) {
      const int c = lane + 64 * k;
      const bool v = c < a.C && c < L;
      p[k] = v ? __expf(a.logp[(long)b * a.C + c]) : 0.f;
      float l = 0.f, u = 1.f;
      if (v) {
        l = cat ? clamped_log(p[k]) : a.logp[(long)b * a.C + c];
        u = (!cat || (p[k] > kPEps && p[k] < 1.f - kPEps)) ? 1.f : 0.f;
      }
      gh[k] = -(l + u);
      S += p[k] * gh[k];
    }
    if (a.d_ent) S = wave_sum(S);
    const long t = (a.d_ce && a.target) ? a.target[b] : (long)a.ignore;
    const long act = (a.d_logp_a && a.action) ? a.action[b] : -1;
    float pa = 0.f;
    if (act >= 0 && cat) {
#pragma unroll
      for (int k = 0; k < kVpl; ++k)
        if (lane + 64 * k == act) pa = p[k];
      pa = wave_max(pa);
    }
    const float ua = (!cat || (pa > kPEps && pa < 1.f - kPEps)) ? 1.f : 0.f;
#pragma unroll
    for (int k = 0; k < kVpl; ++k) {
      const int c = lane + 64 * k;
      if (c >= a.C) continue;
      float g = 0.f;
      if (c < L) {
        if (t != a.ignore) g += a.d_ce[0] * (p[k] - (c == t ? 1.f : 0.f));
        if (act >= 0) g += a.d_logp_a[b] * ua * ((c == act ? 1.f : 0.f) - p[k]);
        if (a.d_ent) g += a.d_ent[b] * p[k] * (gh[k] - S);
      }
      a.dlogit[(long)b * a.ldd + c] = g;
    }
  }
}

}  // namespace

extern "C" int dasa_policy_head_fwd(const float* logit, int64_t ld, const int32_t* cand_len, const int64_t* target,
                                    int32_t B, int32_t C, int32_t mode, int32_t ignore_index, uint64_t seed,
                                    float* logp, float* ce_sum, float* ent, float* logp_a, int64_t* action,
                                    float* ws, void* stream) {
  if (B <= 0) return 0;
  if (C <= 0 || C > 64 * kVpl || ld < C || !logit || !cand_len || !logp || !ce_sum || !ws)
    return (int)hipErrorInvalidValue;
  if (mode != DASA_POLICY_TEACHER && mode != DASA_POLICY_ARGMAX && mode != DASA_POLICY_SAMPLE &&
      mode != DASA_POLICY_FORCED && mode != DASA_POLICY_SAMPLE_ARGMAX)
    return (int)hipErrorInvalidValue;
  if (mode != DASA_POLICY_TEACHER && !action) return (int)hipErrorInvalidValue;
  // a captured sampled step draws fresh actions on every replay: the seed is re-keyed by the device
  // seed source recorded at capture (dasa_set_seed_source), as the dropout kernels do
  PolicyFwd a{logit, (long)ld, cand_len, target, logp, ce_sum, ent, logp_a, action, ws, B, C, mode, ignore_index,
              seed, mode == DASA_POLICY_SAMPLE ? dasa_seed_src_host() : nullptr};
  const int waves = B < 16 ? B : 16;
  hipLaunchKernelGGL(policy_head_fwd_kernel, dim3(1), dim3(64 * waves), 0, (hipStream_t)stream, a);
  DASA_CHECK_LAUNCH();
  return 0;
}

extern "C" int dasa_policy_head_bwd(const float* logp, const int32_t* cand_len, const int64_t* target,
                                    const int64_t* action, const float* ent, const float* d_ce,
                                    const float* d_logp_a, const float* d_ent, float* dlogit, int64_t ldd,
                                    int32_t B, int32_t C, int32_t mode, int32_t ignore_index, void* stream) {
  if (B <= 0 || C <= 0) return 0;
  if (C > 64 * kVpl || ldd < C || !logp || !cand_len || !dlogit || (d_ent && !ent)) return (int)hipErrorInvalidValue;
  if (mode < DASA_POLICY_TEACHER || mode > DASA_POLICY_SAMPLE_ARGMAX) return (int)hipErrorInvalidValue;
  PolicyBwd a{logp, cand_len, target, action, ent, d_ce, d_logp_a, d_ent, dlogit, (long)ldd, B, C, ignore_index,
              mode};
  const int waves = B < 16 ? B : 16;
  const int blocks = (B + waves - 1) / waves;
  hipLaunchKernelGGL(policy_head_bwd_kernel, dim3(blocks < 1024 ? blocks : 1024), dim3(64 * waves), 0,
                     (hipStream_t)stream, a);
  DASA_CHECK_LAUNCH();
  return 0;
}
