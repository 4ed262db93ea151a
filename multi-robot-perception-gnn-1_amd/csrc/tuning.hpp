// tuning.hpp — launch knobs shared by the kernel files (defaults = the measured optima;
// mrp_tuning_set changes them for lab sweeps).
#pragma once

namespace mrp_host {

// Launch geometry knobs (defaults = the measured optima; mrp_tuning_set changes them for lab sweeps).
struct Tuning {
  int fwd_lo = 16, fwd_hi = 64, fwd_cap = 16;  // film_fwd: lanes per plane in [lo, hi], <= cap channels
  int fwd_vec2_below = 0;  // film_fwd: 8-byte slices for planes of fewer than this many pixels (lab knob)
  // film_fwd_regular: whole planes, 32 lanes each (k-NN(4) N=16 C=1024 16x16, B=8: 54.1 us against
  // 57.0 us split over 2 workgroups with 32 lanes; tools/sweep_geometry.py)
  int fwd_regular_split = 0;
  int fwd_regular_lo = 32, fwd_regular_hi = 32, fwd_regular_cap = 16;
  // film_bwd_fused (N <= 8): at most 16 channels per workgroup — at 8x8 planes (8 lanes per plane)
  // two-wave workgroups: configs[3] 24.3 vs 25.6 us with 8 channels, configs[2] 54.7-54.9 vs 55.2
  // (tools/sweep_geometry.py smallbwd; 32 channels: 67.2 vs 60.8 us at C=1280 in round 1); 32x32
  // planes are unaffected (2 channels of 128 lanes)
  int bwd_fused_lo = 8, bwd_fused_hi = 128, bwd_fused_cap = 16;
  // film_bwd_fused: prefetch both slices when a lane owns exactly two — unless a grad_x base is given
  // (2): the base rows are then prefetched instead (configs[1] 217.7 -> 189.9 us with the base,
  // tools/exp_bwd_dxb.py); 1: always, 0: never
  int bwd_pre2 = 2;
  int bwd_regular_vec = 2, bwd_regular_lanes = 16;              // film_bwd_regular (N > 8, k-NN)
  // film_bwd_mfma (Gram and grad_x on the matrix cores; P % 64 == 0, 16-byte aligned operands) for
  // graphs of 9..16 nodes: regular (k-NN; 0 = film_bwd_regular) and complete (0 = film_bwd_dx + the
  // Gram pass: 239.9 vs 90.5 us at B=8 N=16 C=1024 16x16, 65.1 vs 49.4 at B=32 N=12 C=512 8x8,
  // tools/exp_bwd_complete16.py).  Complete graphs of <= 8 nodes keep film_bwd_fused (the matrix-core
  // form, two channels per 16-row block, measured slower there: 30.9 vs 25.7 us at configs[3],
  // 159 vs 143 at [1]; removed in round 3)
  int bwd_regular_mfma = 1;
  int bwd_complete_mfma = 1;
  int bwd_mfma_cpw = 2;  // film_bwd_mfma: 16-row blocks per wave (1 or 2)

  // split-bf16 compress forward / data gradient (compress_split.hip): -1 per shape, 7 (256-row
  // workgroups on 16x16x32 MFMAs, where M % 256 == 0) or 2 (128-row workgroups on 32x32x16)
  int gemm_split = -1;
  // mrp_edge_encoder_fwd_split (encoder_split.hip): -1 per shape, 1 = 4 waves, 3 = 8 waves per workgroup
  int edge_split_v = -1;
  int edge_allx = 1;  // mrp_edge_encoder_fwd_split: all hidden blocks before z where they fit LDS (0 off)
  // split-bf16 weight-gradient (NT) kernel: 4 (the default where C >= 1024) the compress weight gradient
  // with dy split once into a packed image (split_rows + gemm_nt_psa) where the image fits 32-bit
  // offsets, else (and for the encoder's products) 3 (the default below C = 1024): the 32-k-stage form
  // on 16x16x32 MFMAs splitting both operands
  int split_nt = -1;
  // split-bf16 GEMMs' tile order (compress_split.hip tile_of): runs of this many 256-row tiles, m
  // fastest (0: all, round 4's order).  Forward / data gradient 4 (configs[3] 1.4-1.8 % faster, the
  // others flat; tools/ab_gemm.py knob:gemm_group=0,4); weight gradient 0 (4 measured 1.6-2.7 % slower
  // at configs[2] and [3])
  int gemm_group = 4;
  int nt_group = 0;
  // mrp_edge_encoder_bwd_fused, given W2^T's packed image: 2 = both products read their A operand
  // pre-split (W2^T's image; dz^T written as an image by dzT_pack), 1 = only W2^T's, 0 = neither
  int enc_bwd_psa = 2;
  int enc_s1 = 0, enc_s2 = 0;  // mrp_edge_encoder_bwd_fused: split counts of its two products (0: planner)
};
Tuning& tuning();

}  // namespace mrp_host
