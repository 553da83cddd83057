// Parameter block for the fp32 attention kernels (csrc/attn_f32.hip), filled by the host binding (csrc/bind.cpp).
// Tensors are [B, S, H, 64] fp32 views with the head dim contiguous; strides in elements.
#pragma once
#include <stdint.h>

struct AttnF32Params {
  const float* q;
  const float* k;
  const float* v;
  const float* o;     // bwd: forward output
  const float* dout;  // bwd: output gradient
  float* o_out;       // fwd output
  float* lse;         // [B, H, Sq]: fwd writes, bwd reads
  float* delta;       // [B, H, Sq]: rowsum(dO * O), written by the bwd pre-pass
  float* dq;
  float* dk;
  float* dv;
  float* dlut;        // [H, Sq + Sk - 1] (bwd, accumulated with atomics; zeroed by the host)
  const uint8_t* kpm; // [B, Sk] 1 = attend
  const float* lut;   // [H, Sq + Sk - 1] additive bias by relative position (key - row + Sq - 1)
  long q_sb, q_ss, q_sh;
  long k_sb, k_ss, k_sh;
  long v_sb, v_ss, v_sh;
  long o_sb, o_ss, o_sh;
  long do_sb, do_ss, do_sh;
  long dq_sb, dq_ss, dq_sh;
  long dk_sb, dk_ss, dk_sh;
  long dv_sb, dv_ss, dv_sh;
  int B, H, Sq, Sk;
  float scale;
  int causal;
  int causal_off;  // Sk - Sq
  float p_drop;
  uint32_t seed;
  uint32_t thr;    // 16-bit keep threshold (ops/rng.py threshold16)
};
