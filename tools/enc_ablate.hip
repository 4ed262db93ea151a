// Kernel lab (not product code): ablations of the shared-hidden split-bf16 encoder forward
// (encoder_split.hip, encoder2_body's ABL bits: 1 = W2 fragments from registers, no loads; 2 = no
// hidden-layer MFMAs; 4 = no barrier per round; 8 = no z MFMAs; 16 = no hidden-fragment LDS reads;
// 32 = no z stores; 64 = no ReLU/split/LDS store of X) at the BASELINE encoder shapes, timed
// with hipEvents.  Outputs of ablated runs are garbage by design.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include tools/enc_ablate.hip -o tools/bin/enc_ablate
#include "../multi-robot-perception-gnn-1_amd/csrc/encoder_split.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

namespace mrp_host {
Tuning& tuning() {
  static Tuning t;
  return t;
}
}  // namespace mrp_host

namespace mrp_x6 {
template <int CB, int NWV, int ABL>
__global__ void __launch_bounds__(64 * NWV) abl_kernel(FwdArgs a) {
#if defined(__HIP_DEVICE_COMPILE__)
  encoder2_body<CB, NWV, ABL>(a);
#endif
}
}  // namespace mrp_x6
using namespace mrp_x6;

template <int CB, int NWV, int ABL>
float run(FwdArgs a, int iters, hipStream_t st) {
  const int grid = ((a.E + 31) / 32) * ((2 * a.C / 32 + NWV * CB - 1) / (NWV * CB));
  const size_t lds = (size_t)2 * NWV * 6 * 64 * 16;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  std::vector<float> ts;
  for (int r = 0; r < 7; ++r) {
    hipEventRecord(e0, st);
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((abl_kernel<CB, NWV, ABL>), dim3(grid), dim3(64 * NWV), lds, st, a);
    hipEventRecord(e1, st);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ts.push_back(ms * 1000 / iters);
  }
  std::sort(ts.begin(), ts.end());
  return ts[3];
}

int main(int argc, char** argv) {
  const int E = argc > 1 ? atoi(argv[1]) : 1792, C = argc > 2 ? atoi(argv[2]) : 512;
  float *pose, *w1, *b1, *w2, *b2, *z;
  void* pk;
  hipMalloc(&pose, (size_t)E * 9 * 4);
  hipMalloc(&w1, (size_t)C * 9 * 4);
  hipMalloc(&b1, (size_t)C * 4);
  hipMalloc(&w2, (size_t)2 * C * C * 4);
  hipMalloc(&b2, (size_t)2 * C * 4);
  hipMalloc(&z, (size_t)E * 2 * C * 4);
  hipMalloc(&pk, mrp_edge_encoder_pack_bytes(C));
  hipMemset(pose, 0, (size_t)E * 9 * 4);
  hipMemset(w1, 0, (size_t)C * 9 * 4);
  hipMemset(b1, 0, (size_t)C * 4);
  hipMemset(w2, 0, (size_t)2 * C * C * 4);
  hipStream_t st;
  hipStreamCreate(&st);
  mrp_edge_encoder_pack(w1, b1, w2, C, pk, st);
  FwdArgs a = {};
  a.pose = pose;
  a.packed = static_cast<const u4*>(pk);
  a.b2 = b2;
  a.z = z;
  a.E = E;
  a.C = C;
  const int it = 50;
  printf("E=%d C=%d  cb1_w8: full %.2f | noW2load %.2f | noX %.2f | nobar %.2f | noZmfma %.2f | noW2+noZ %.2f | "
         "all four off %.2f | +no hp reads %.2f | +no z stores %.2f | +no X split/store %.2f | everything off %.2f us\n",
         E, C, run<1, 8, 0>(a, it, st), run<1, 8, 1>(a, it, st), run<1, 8, 2>(a, it, st), run<1, 8, 4>(a, it, st),
         run<1, 8, 8>(a, it, st), run<1, 8, 9>(a, it, st), run<1, 8, 15>(a, it, st), run<1, 8, 31>(a, it, st),
         run<1, 8, 47>(a, it, st), run<1, 8, 79>(a, it, st), run<1, 8, 127>(a, it, st));
  return 0;
}
