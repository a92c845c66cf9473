// Internal interface between the bi-LSTM entry points (lstm.hip) and the persistent kernels
// (lstm_persist.hip). Not part of the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

bool bilstm_persist_ok(int B, int H);       // backward: B <= 32
bool bilstm_persist_fwd_ok(int B, int H);   // forward: B <= 32, or B <= 192 at H = 1024 (6 batch tiles)
bool bilstm_fwd_x6_on();                    // dasa_bilstm_fwd_x6 (the bf16x6 recurrent product)
int bilstm_persist_fwd(const float* xproj, const float* whh_fwd, const float* whh_bwd, const int32_t* lengths,
                       float* out, float* h_n, float* c_n, float* save_act, float* save_c, int B, int L, int H,
                       float* hbuf, unsigned* sync, hipStream_t st);
int bilstm_persist_bwd(const float* whh_fwd, const float* whh_bwd, const int32_t* lengths, const float* save_act,
                       const float* save_c, const float* dout, const float* dh_n, const float* dc_n, float* dgates,
                       int B, int L, int H, unsigned* sync, hipStream_t st);
