/*
 * mrp_gnn.h — C ABI of the MI355X (gfx950) FiLM-mean message-passing library.
 *
 * This is the drop-in boundary for the GCN aggregation hot path of
 * xjh19971/multi-robot-perception-gnn-1.  The reference executes it as
 *
 *     g.edata['pose_gamma'], g.edata['pose_beta'] = edge_encoder(g.edata['pose'])
 *     g.update_all(edge_udf, node_udf)                 dgl/model/models.py:222-223
 *
 * with edge_udf  m_e   = gamma_e * x_src(e) + beta_e   dgl/model/models.py:210-211
 * and  node_udf  out_v = mean over v's mailbox          dgl/model/models.py:207-208
 * executed by DGL's update_all (gather -> message -> degree bucket -> reduce).
 *
 * Each entry point below replaces the DGL `update_all(edge_udf, node_udf)` call
 * (forward) or its autograd backward; the edge encoder stays a torch Linear stack
 * whose sigmoid output (E, 2C) is consumed *in place* as the interleaved (E, C, 2)
 * gamma/beta tensor that `edge.view(-1, C, 2)` exposes (dgl/model/models.py:154-155).
 *
 * Conventions
 *  - All pointers are device pointers owned by the caller; the library never
 *    allocates, frees or synchronises.  Work is enqueued on `stream`
 *    (a hipStream_t; NULL = the legacy default stream).
 *  - Node features are fp32, node-major: node v's C x P block (P = H*W) starts at
 *    x + v * x_node_stride, channel c's plane at + c * P, contiguous over P.
 *    x_node_stride >= C * P.  (A stride of 2*C*P writes straight into one half of
 *    the torch.cat((h, g_h), 1) buffer, dgl/model/models.py:182.)
 *  - The batched graph is a disjoint union of per-frame graphs (dgl.batch,
 *    dgl/training.py:57-58): graph b owns nodes [graph_off[b], graph_off[b+1]),
 *    at most MRP_MAX_NODES nodes, and every edge stays inside one graph.
 *    Edges are given as CSR by destination: the in-edges of node v occupy
 *    positions [indptr[v], indptr[v+1]) of `src` (global source node id) and
 *    `eid` (row of the (E, C, 2) gamma/beta tensor), in increasing edge-id order
 *    (DGL mailbox order).
 *  - Return value: 0 on success, otherwise a hipError_t value
 *    (hipErrorInvalidValue = 1 for bad shapes/arguments).  No exceptions cross
 *    the ABI.  Stateless and re-entrant.
 */
#ifndef MRP_GNN_H
#define MRP_GNN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MRP_MAX_NODES 16

/* Graph kinds.  MRP_GRAPH_COMPLETE is the reference's only topology (dgl/dataloader.py:88-95):
 * every graph has exactly max_nodes nodes, edges are all ordered pairs u != v, numbered graph by
 * graph in i-major order (edge u->v of graph b is b*n*(n-1) + u*(n-1) + (v < u ? v : v-1)), and
 * node ids are graph by graph.  indptr/src/eid/graph_off are then not read (may be NULL).
 * MRP_GRAPH_CSR is any batch of disjoint graphs described by the CSR arrays.
 *
 * Preconditions the kernels rely on and do not check on the device (the library never reads
 * device memory on the host; RobotGraph.csr() establishes them, and breaking them gives wrong or
 * partially unwritten outputs rather than an error):
 *   - every graph b has graph_off[b+1] - graph_off[b] <= max_nodes nodes;
 *   - every edge's source lies in its destination's graph;
 *   - MRP_GRAPH_REGULAR(k): every node has exactly k in-edges, so node v's CSR row is
 *     [k*v, k*(v+1)) (indptr is then not read by the forward);
 *   - MRP_GRAPH_COMPLETE: the edge numbering below. */
enum mrp_graph_kind {
    MRP_GRAPH_CSR = 0,
    MRP_GRAPH_COMPLETE = 1
};
/* MRP_GRAPH_REGULAR(k): a CSR graph in which every node has exactly k in-edges (k-NN graphs).  The
 * CSR arrays are read as for MRP_GRAPH_CSR; the backward for graphs of more than 8 nodes then keeps
 * one Gram accumulator per edge instead of per node pair (k <= 8).  num_edges must be k*num_nodes.
 * Node v's CSR row is then [k*v, k*(v+1)) by construction (CSR by destination, uniform degree), so
 * the forward does not read indptr. */
#define MRP_GRAPH_REGULAR(k) (((k) << 8) | 2)
#define MRP_GRAPH_IS_REGULAR(kind) (((kind) & 0xff) == 2)
#define MRP_GRAPH_REGULAR_K(kind) ((kind) >> 8)

/* Aggregation modes (the reference's UDF variants). */
enum mrp_agg_mode {
    MRP_AGG_FILM_MEAN = 0, /* mean_e(gamma_e*x_u + beta_e): models.py:207-211          */
    MRP_AGG_FILM_SUM = 1,  /* sum_e(gamma_e*x_u + beta_e)                              */
    MRP_AGG_COPY_MEAN = 2  /* mean_e(x_u), fn.copy_u('image','m'): models.py:225,
                              dgl_models.py:126 ("multi_view_dgl_mean_wofilm")         */
};

/* Flag OR-ed into `mode`: gb holds the edge encoder's pre-sigmoid logits z (the output of its
 * second Linear); the kernels apply gamma/beta = sigmoid(z) while building their tiles (forward)
 * and return d z = d gamma/beta * s (1 - s) (backward).  Fuses the encoder's Sigmoid
 * (dgl/model/models.py:150) into the aggregation. */
#define MRP_AGG_GB_LOGITS 0x100

/*
 * Forward: out[v] = reduce over in-edges e=(u->v) of (gamma_e (.) x[u] + beta_e).
 * Replaces g.update_all(edge_udf, node_udf), dgl/model/models.py:223.
 * Nodes with zero in-degree get zeros (DGL >= 0.5 zero-fill).
 *
 *   x          (num_nodes, C, P) fp32, node stride x_node_stride (elements)
 *   gb         (num_edges, C, 2) fp32 interleaved gamma/beta; may be NULL for COPY_MEAN
 *   indptr     (num_nodes + 1) int32, CSR by destination
 *   src, eid   (num_edges) int32
 *   graph_off  (num_graphs + 1) int32 node offsets of the batched graphs
 *   max_nodes  max_b (graph_off[b+1] - graph_off[b]), 0..MRP_MAX_NODES (host-known)
 *   graph_kind MRP_GRAPH_CSR, MRP_GRAPH_COMPLETE or MRP_GRAPH_REGULAR(k) (see enum mrp_graph_kind)
 *   out        (num_nodes, C, P) fp32, node stride out_node_stride (elements)
 */
int mrp_film_mean_fwd(const float* x, int64_t x_node_stride,
                      const float* gb,
                      const int32_t* indptr, const int32_t* src, const int32_t* eid,
                      const int32_t* graph_off, int32_t num_graphs, int32_t max_nodes,
                      int32_t graph_kind, int32_t num_nodes, int32_t num_edges,
                      int32_t C, int32_t P, int32_t mode,
                      float* out, int64_t out_node_stride,
                      void* stream);

/*
 * torch.cat((x, update_all(...)), 1) in one pass (dgl/model/models.py:181-182, 186-188): as
 * mrp_film_mean_fwd, but `cat` is the (num_nodes, 2C, P) concatenation buffer (node stride
 * cat_node_stride >= 2*C*P): x is written to channels [0, C) and the aggregate to [C, 2C).  The
 * kernel stores the slices of x it already holds in registers, so x is read once instead of twice.
 */
int mrp_film_mean_cat_fwd(const float* x, int64_t x_node_stride,
                          const float* gb,
                          const int32_t* indptr, const int32_t* src, const int32_t* eid,
                          const int32_t* graph_off, int32_t num_graphs, int32_t max_nodes,
                          int32_t graph_kind, int32_t num_nodes, int32_t num_edges,
                          int32_t C, int32_t P, int32_t mode,
                          float* cat, int64_t cat_node_stride,
                          void* stream);

/*
 * Backward of mrp_film_mean_fwd (the autograd of models.py:207-211 through DGL's
 * gather/mailbox, which the reference gets from torch autograd).  With s_v the
 * reduce scale (1/deg v for the mean modes, 1 for SUM) and G = grad_out:
 *
 *   grad_x[u]      = sum_{e=(u->v)} s_v * gamma_e (.) G[v]          (gamma = 1 for COPY)
 *   grad_gb[e,c,0] = s_v * sum_p x[u,c,p] * G[v,c,p]                (d gamma_e)
 *   grad_gb[e,c,1] = s_v * sum_p G[v,c,p]                           (d beta_e)
 *
 * grad_x (node stride gx_node_stride) and grad_gb ((num_edges, C, 2), interleaved
 * like gb) may each be NULL to skip that output.  For COPY_MEAN grad_gb is zero-filled.
 * grad_x_base (node stride base_node_stride, may be NULL) is added to grad_x: the backward of
 * torch.cat((x, out), 1) (dgl/model/models.py:182) passes the first half of the concatenation's
 * gradient here and the second half as grad_out, so x's total gradient is one pass.
 * Deterministic: no atomics; each output element is written by exactly one lane.
 */
int mrp_film_mean_bwd(const float* grad_out, int64_t g_node_stride,
                      const float* x, int64_t x_node_stride,
                      const float* gb,
                      const int32_t* indptr, const int32_t* src, const int32_t* eid,
                      const int32_t* graph_off, int32_t num_graphs, int32_t max_nodes,
                      int32_t graph_kind, int32_t num_nodes, int32_t num_edges,
                      int32_t C, int32_t P, int32_t mode,
                      float* grad_x, int64_t gx_node_stride,
                      const float* grad_x_base, int64_t base_node_stride,
                      float* grad_gb,
                      void* stream);

/*
 * Epilogue of the aggregation, for the layer compositions around update_all.  With a = the
 * aggregate of destination v (as mrp_film_mean_fwd computes it), the forward writes
 *
 *   out[v] = agg_scale * a + self_scale * x[v] + x0_scale * x0[v]
 *
 * evaluated left to right in fp32 (each product rounded, then each sum; a scale of 1 is exact), and
 * if xcopy != NULL also stores x[v] at xcopy + v * xcopy_node_stride.  Uses:
 *   - plain aggregation:  {1, 0, NULL, 0, 0, NULL, 0} (what a NULL epilogue pointer means);
 *   - residual h = g_h + h (dgl/model/dgl_models.py:36-37): agg_scale 1, self_scale 1 — x[v] is
 *     already in registers, so this costs no traffic;
 *   - initial-feature mix (GCN2-style, (1 - alpha) * a + alpha * x0; not in the reference, parity
 *     unpinned): agg_scale 1 - alpha, x0 = the first layer's input, x0_scale alpha;
 *   - torch.cat((x, a), 1) (dgl/model/models.py:182): xcopy = the first half of the concatenation
 *     buffer (mrp_film_mean_cat_fwd is this with out = its second half).
 * The backward (mrp_film_mean_bwd_ex) reads agg_scale and self_scale: grad_out reaches the
 * aggregation scaled by agg_scale, and self_scale * grad_out[u] is added to grad_x[u].  The
 * gradient of x0 is x0_scale * grad_out (an elementwise product the caller forms); x0 and xcopy
 * are not read by the backward.
 */
typedef struct mrp_agg_epilogue {
    float agg_scale;
    float self_scale;
    const float* x0;
    int64_t x0_node_stride;
    float x0_scale;
    float* xcopy;
    int64_t xcopy_node_stride;
} mrp_agg_epilogue;

/* mrp_film_mean_fwd with an epilogue (NULL: plain).  x0 and xcopy rows use the node ids of x. */
int mrp_film_mean_fwd_ex(const float* x, int64_t x_node_stride,
                         const float* gb,
                         const int32_t* indptr, const int32_t* src, const int32_t* eid,
                         const int32_t* graph_off, int32_t num_graphs, int32_t max_nodes,
                         int32_t graph_kind, int32_t num_nodes, int32_t num_edges,
                         int32_t C, int32_t P, int32_t mode,
                         float* out, int64_t out_node_stride,
                         const mrp_agg_epilogue* epilogue,
                         void* stream);

/* mrp_film_mean_bwd for a forward run with `epilogue` (NULL: plain; see mrp_agg_epilogue).
 * workspace: reserved (NULL/0 allowed; mrp_film_mean_bwd_workspace returns 0): ABI 11's plane-split
 * k-NN backward that used it measured slower than whole planes and was removed in ABI 12. */
int mrp_film_mean_bwd_ex(const float* grad_out, int64_t g_node_stride,
                         const float* x, int64_t x_node_stride,
                         const float* gb,
                         const int32_t* indptr, const int32_t* src, const int32_t* eid,
                         const int32_t* graph_off, int32_t num_graphs, int32_t max_nodes,
                         int32_t graph_kind, int32_t num_nodes, int32_t num_edges,
                         int32_t C, int32_t P, int32_t mode,
                         float* grad_x, int64_t gx_node_stride,
                         const float* grad_x_base, int64_t base_node_stride,
                         float* grad_gb,
                         const mrp_agg_epilogue* epilogue,
                         void* workspace, int64_t workspace_bytes,
                         void* stream);

/* Bytes of workspace mrp_film_mean_bwd_ex can use for these graph/feature sizes (0: none needed;
 * always 0 since ABI 12). */
int64_t mrp_film_mean_bwd_workspace(int32_t num_graphs, int32_t max_nodes, int32_t graph_kind,
                                    int32_t C, int32_t P);

/*
 * The layer's 1x1 compress convolution and its gradients, fp32 on the matrix cores (exact fp32
 * products, v_mfma_f32_32x32x2_f32), without the concatenation (dgl/model/models.py:163-165,181-184,
 * 186-189: h = conv(torch.cat((x, a), 1)) with conv = nn.Conv2d(2C, C, kernel_size=1)).  W is the
 * conv weight (C, 2C) row-major (nn.Conv2d's (C, 2C, 1, 1)); x and a are the two halves of the
 * concatenation as separate node-major tensors (any node strides, e.g. the two halves of one cat
 * buffer).  Requirements (else hipErrorNotSupported): C % 32 == 0, P % 4 == 0, node strides % 4 == 0,
 * every tensor 16-byte aligned, each operand's node range addressable with 31-bit byte offsets.
 *
 * mrp_compress_fwd:       y[n] = W[:, :C] x[n] + W[:, C:] a[n] + bias      (bias (C) may be NULL)
 * mrp_compress_bwd_data:  gx[n] = W[:, :C]^T gy[n],  ga[n] = W[:, C:]^T gy[n]
 *                         wt = W^T (2C, C), from mrp_compress_weight_transpose
 * mrp_compress_bwd_weight: gw = sum_n gy[n] [x[n]; a[n]]^T (C, 2C),  gbias = sum_{n,p} gy (may be
 *                         NULL); split over the node-pixel axis into workspace (>=
 *                         mrp_compress_bwd_weight_workspace bytes for the largest of the three node
 *                         strides, 16-byte aligned; 0 = none needed), partial sums added in a fixed
 *                         order (deterministic).  Also needs P % 32 == 0 and C % 8 == 0.
 */
int mrp_compress_fwd(const float* x, int64_t x_node_stride, const float* a, int64_t a_node_stride,
                     int32_t num_nodes, int32_t C, int32_t P, const float* w, const float* bias,
                     float* y, int64_t y_node_stride, void* stream);
int mrp_compress_weight_transpose(const float* w, float* wt, int32_t C, void* stream);
int mrp_compress_bwd_data(const float* gy, int64_t gy_node_stride, int32_t num_nodes, int32_t C, int32_t P,
                          const float* wt, float* gx, int64_t gx_node_stride, float* ga, int64_t ga_node_stride,
                          void* stream);
int64_t mrp_compress_bwd_weight_workspace(int32_t num_nodes, int32_t C, int32_t P, int64_t max_node_stride);
int mrp_compress_bwd_weight(const float* gy, int64_t gy_node_stride, const float* x, int64_t x_node_stride,
                            const float* a, int64_t a_node_stride, int32_t num_nodes, int32_t C, int32_t P,
                            float* gw, float* gbias, void* workspace, int64_t workspace_bytes, void* stream);

/*
 * The compress forward and data gradient on the bf16 matrix cores at fp32 accuracy
 * (compress_split.hip): the same products as mrp_compress_fwd / mrp_compress_bwd_data, each fp32
 * operand split exactly into three bf16 parts and each product the sum of the six partial products
 * whose omitted terms are below 2^-25 of it (error against float64 at or below an fp32 GEMM's).  The
 * weight operand is split and laid out once per weight version:
 *   mrp_compress_split_pack_bytes(M, K)   bytes of a packed M x K operand (0 unless M % 32 == 0, K % 16 == 0)
 *   mrp_compress_split_pack(w, ld, transpose, M, K, packed)
 *                                         A = w (M x K row-major, row stride ld) or, transpose != 0,
 *                                         A = w^T (w: K x M row-major, row stride ld) -> packed (16-byte aligned)
 *   mrp_compress_fwd_split                y = W [x; agg] + b with packed = pack(w, 2C, 0, C, 2C)
 *   mrp_compress_bwd_data_split           [gx; gagg] = W^T gy with packed = pack(w, 2C, 1, 2C, C)
 * Arguments otherwise as mrp_compress_fwd / mrp_compress_bwd_data.  Requirements (else
 * hipErrorNotSupported): C % 32 == 0, P % 4 == 0, x / agg / gy 16-byte aligned with node strides % 4 == 0.
 */
int64_t mrp_compress_split_pack_bytes(int32_t M, int32_t K);
int mrp_compress_split_pack(const float* w, int64_t ld, int32_t transpose, int32_t M, int32_t K, void* packed,
                            void* stream);
int mrp_compress_fwd_split(const float* x, int64_t x_node_stride, const float* agg, int64_t agg_node_stride,
                           int32_t num_nodes, int32_t C, int32_t P, const void* packed_w, const float* bias, float* y,
                           int64_t y_node_stride, void* stream);
int mrp_compress_bwd_data_split(const float* gy, int64_t gy_node_stride, int32_t num_nodes, int32_t C, int32_t P,
                                const void* packed_wt, float* gx, int64_t gx_node_stride, float* gagg,
                                int64_t gagg_node_stride, void* stream);

/*
 * The compress weight gradient (mrp_compress_bwd_weight's products) on the split-bf16 matrix cores:
 * both operands are activations, split in the kernel on their way into LDS; K = num_nodes P split over
 * workgroups into partial tiles summed in a fixed order (deterministic).  Workspace: device buffer of
 * mrp_compress_bwd_weight_split_workspace(num_nodes, C, P) bytes (0: none needed).  Requirements (else
 * hipErrorNotSupported): C % 64 == 0, P % 32 == 0, 16-byte aligned operands, node strides % 4 == 0.
 */
int64_t mrp_compress_bwd_weight_split_workspace(int32_t num_nodes, int32_t C, int32_t P);
int mrp_compress_bwd_weight_split(const float* gy, int64_t gy_node_stride, const float* x, int64_t x_node_stride,
                                  const float* a, int64_t a_node_stride, int32_t num_nodes, int32_t C, int32_t P,
                                  float* gw, float* gbias, void* workspace, int64_t workspace_bytes, void* stream);

/*
 * First layer of the edge encoder, dgl/model/models.py:147-148:  h = relu(pose W1^T + b1).
 *   pose (num_edges, 9), w1 (C, 9) (nn.Linear weight layout), b1 (C) -> h (num_edges, C), fp32.
 * The second Linear is mrp_edge_logits_fwd and its Sigmoid is fused into the aggregation
 * (MRP_AGG_GB_LOGITS).
 */
int mrp_edge_hidden_fwd(const float* pose, const float* w1, const float* b1,
                        int32_t num_edges, int32_t C, float* h, void* stream);

/*
 * Second layer of the edge encoder before its Sigmoid, dgl/model/models.py:149:
 *   z = h W2^T + b2,  h (num_edges, C), w2 (2C, C) (nn.Linear weight layout), b2 (2C) -> z (num_edges, 2C)
 * fp32 on the matrix cores (exact fp32 products), the bias added in the epilogue.  z is the logits
 * tensor the aggregation reads with MRP_AGG_GB_LOGITS.  Requirements (else hipErrorNotSupported):
 * C % 32 == 0, h and w2 16-byte aligned, h and w2 under 2^31 bytes.
 */
int mrp_edge_logits_fwd(const float* h, int32_t num_edges, int32_t C, const float* w2, const float* b2,
                        float* z, void* stream);

/*
 * The edge encoder before its Sigmoid in one launch (dgl/model/models.py:146-149),
 *   z = relu(pose W1^T + b1) W2^T + b2     pose (num_edges, 9), w1 (C, 9), b1 (C), w2 (2C, C), b2 (2C),
 * at fp32 accuracy on the bf16 matrix cores (encoder_split.hip): every fp32 operand is
 * split exactly into three bf16 parts and each product is the sum of the six partial products whose
 * omitted terms are below 2^-25 of it (error against float64 at or below an fp32 GEMM's); the hidden
 * layer is computed on the matrix cores too (b1 as a tenth input of value 1.0) and never written.
 * The weights are split and laid out once per weight version:
 *   mrp_edge_encoder_pack_bytes(C)  bytes of the packed image (0 if C <= 0 or C % 32 != 0)
 *   mrp_edge_encoder_pack           w1 (C, 9), b1 (C), w2 (2C, C) -> packed (16-byte aligned device buffer)
 *   mrp_edge_encoder_fwd_split      z = relu(pose W1^T + b1) W2^T + b2 from pose (E, 9), the packed image
 *                                   and b2 (2C, or NULL) -> z (E, 2C)
 * Requirements (else hipErrorNotSupported): C % 32 == 0 and a packed image below 2^31 bytes (the
 * kernel addresses it with 32-bit offsets: C <= 13344).  The z accumulation keeps the a0 b0 products
 * apart from the five small ones (two accumulators per output, summed once).  Used for inference;
 * training keeps h for its backward and runs mrp_edge_hidden_fwd + mrp_edge_logits_fwd.
 */
int64_t mrp_edge_encoder_pack_bytes(int32_t C);
int mrp_edge_encoder_pack(const float* w1, const float* b1, const float* w2, int32_t C, void* packed, void* stream);
int mrp_edge_encoder_fwd_split(const float* pose, const void* packed, const float* b2, int32_t num_edges, int32_t C,
                               float* z, void* stream);

/*
 * The encoder's training path on the split-bf16 matrix cores (replaces mrp_edge_hidden_fwd +
 * mrp_edge_logits_fwd forward and the two library GEMMs of the backward, dgl/model/models.py:146-149
 * under dgl/training.py:208-210's loss.backward()):
 *   mrp_edge_encoder_fwd_split_train   as mrp_edge_encoder_fwd_split (shared-hidden form), and also
 *                                      h^T = relu(pose W1^T + b1)^T, (C, E) rows of hT_stride >= E floats
 *   mrp_edge_encoder_bwd_prep          dzT (2C, E) rows of dzT_stride >= E = dz^T (E % 4 == 0, C even,
 *                                      16-byte aligned, dzT_stride % 4 == 0; else hipErrorNotSupported)
 *   mrp_edge_encoder_bwd_split         dh^T (C, E) = W2^T dz^T and dW2 (2C, C) = dz^T h on the split-bf16
 *                                      weight-gradient kernel (either output may be NULL), with db2 (2C) =
 *                                      column sums of dz taken on the dW2 product (NULL, or dw2 non-NULL);
 *                                      w2T = W2^T (C, 2C) row-major; dzT and hT with row stride E;
 *                                      workspace: _split_workspace(E, C) bytes (0 if none is needed) —
 *                                      the two products may be issued as two calls on two streams, each
 *                                      with its own workspace
 *   mrp_edge_encoder_bwd_t             dpre = dh^T (.) [h^T > 0]: dw1 (C, 9) = dpre pose, db1 (C) = row sums
 *                                      (either may be NULL); workspace: _t_workspace(E, C) bytes
 *   mrp_edge_encoder_bwd_fused         the whole backward of the encoder's parameters in three launches
 *                                      on one stream: dz^T; dh^T and dW2 as ONE launch of both split-K
 *                                      products; a reduction that sums their partial tiles, applies the
 *                                      ReLU mask and forms dW1 / db1 (dh^T never written).  dw1, db1,
 *                                      dw2, db2 all required (no dpose); w2T_packed: NULL, or W2^T's
 *                                      packed split image (mrp_compress_split_pack(w2, C, 1, C, 2C), 16-byte
 *                                      aligned), which the dh^T product then reads instead of splitting
 *                                      w2T in every workgroup, and dz^T is then written as a packed image
 *                                      for the dW2 product too (same products, same order: dW1, db1 and
 *                                      dW2 bit-identical to the split form; db2 summed per 64-edge block);
 *                                      workspace: _fused_workspace(E, C) bytes
 *   mrp_edge_encoder_bwd_pose          the pose gradient (the encoder's input, wanted only when poses
 *                                      require grad): dpose (E, 9) = dpre^T W1 with dpre as for _bwd_t;
 *                                      any E, C; workspace: _pose_workspace(E, C) bytes (0: none needed)
 * Requirements of _bwd_split and _bwd_fused (else hipErrorNotSupported): E % 32 == 0, C % 32 == 0,
 * 16-byte aligned operands.  Shapes outside them run the same kernels on zero-padded operands
 * (encoder.py, EdgeEncoderPaddedFunction: E and C rounded up to 32, zero weight rows and columns, zero
 * gradient rows — every padded term a product with an exact zero).  All sums in a fixed order:
 * deterministic.
 */
int mrp_edge_encoder_fwd_split_train(const float* pose, const void* packed, const float* b2, int32_t num_edges,
                                     int32_t C, float* z, float* hT, int64_t hT_stride, void* stream);
int mrp_edge_encoder_bwd_prep(const float* dz, int32_t num_edges, int32_t C, float* dzT, int64_t dzT_stride,
                              void* stream);
int64_t mrp_edge_encoder_bwd_split_workspace(int32_t num_edges, int32_t C);
int mrp_edge_encoder_bwd_split(const float* dz, const float* dzT, const float* w2T, const float* hT,
                               int32_t num_edges, int32_t C, float* dhT, float* dw2, float* db2, void* workspace,
                               int64_t workspace_bytes, void* stream);
int64_t mrp_edge_encoder_bwd_fused_workspace(int32_t num_edges, int32_t C);
int mrp_edge_encoder_bwd_fused(const float* dz, const float* w2T, const void* w2T_packed, const float* hT,
                               const float* pose, int32_t num_edges, int32_t C, float* dw1, float* db1, float* dw2,
                               float* db2, void* workspace, int64_t workspace_bytes, void* stream);
int64_t mrp_edge_encoder_bwd_t_workspace(int32_t num_edges, int32_t C);
int mrp_edge_encoder_bwd_t(const float* dhT, int64_t dhT_stride, const float* hT, int64_t hT_stride,
                           const float* pose, int32_t num_edges, int32_t C, float* dw1, float* db1, void* workspace,
                           int64_t workspace_bytes, void* stream);
int64_t mrp_edge_encoder_bwd_pose_workspace(int32_t num_edges, int32_t C);
int mrp_edge_encoder_bwd_pose(const float* dhT, int64_t dhT_stride, const float* hT, int64_t hT_stride,
                              const float* w1, int32_t num_edges, int32_t C, float* dpose, void* workspace,
                              int64_t workspace_bytes, void* stream);

/*
 * Backward of the edge encoder's reductions (dgl/model/models.py:147-149), run after the two
 * library GEMMs of its backward (dh = dz W2, dW2 = dz^T h):
 *   db2[j]    = sum_e dz[e, j]                              (dz: (E, 2C), the logits' gradient that
 *                                                            mrp_film_mean_bwd writes with MRP_AGG_GB_LOGITS)
 *   dw1[k, i] = sum_e dh[e, k] * [h[e, k] > 0] * pose[e, i] (dh, h: (E, C); pose (E, 9); dw1 (C, 9))
 *   db1[k]    = sum_e dh[e, k] * [h[e, k] > 0]
 * workspace: device buffer of mrp_edge_encoder_bwd_workspace(E, C) bytes.  Outputs may be NULL.
 * Deterministic (fixed summation order, no atomics).
 */
int64_t mrp_edge_encoder_bwd_workspace(int32_t num_edges, int32_t C);
int mrp_edge_encoder_bwd(const float* dz, const float* dh, const float* h, const float* pose,
                         int32_t num_edges, int32_t C, float* db2, float* dw1, float* db1,
                         float* workspace, void* stream);

/*
 * Per-frame robot graphs built on the device (dgl/dataloader.py:88-122 with the relative pose of
 * dgl/utils.py:54-77), for a batch of num_graphs frames of n robots each (n <= MRP_MAX_NODES).
 *
 *   poses      (num_graphs * n, 7) fp32 rows (tx, ty, tz, qx, qy, qz, qw), graph by graph
 *   knn_k      0: complete graphs, the reference topology: all ordered pairs u != v, edges numbered
 *                 graph by graph i-major (the MRP_GRAPH_COMPLETE numbering), E = num_graphs*n*(n-1);
 *              k (1 <= k < n): k-NN graphs: destination v's sources are the k robots u != v with the
 *                 smallest |t_u - t_v| (float64, ties to the lower index), edges numbered
 *                 destination-major with sources ascending, E = num_graphs*n*k (MRP_GRAPH_REGULAR(k))
 *   edge_pose  (E, 9) fp32: cal_relative_pose(pose[src e], pose[dst e]), bit-identical to the
 *              reference's float32 arithmetic
 *   indptr     (num_graphs*n + 1), src (E), eid (E): CSR by destination, in-edges by increasing
 *              edge id; graph_off (num_graphs + 1) — the graph arguments of the aggregation calls
 * Any output pointer may be NULL to skip it.  Returns hipErrorInvalidValue for n > MRP_MAX_NODES,
 * k >= n or sizes beyond int32.
 */
int mrp_frame_graph_build(const float* poses, int32_t num_graphs, int32_t n, int32_t knn_k,
                          float* edge_pose, int32_t* indptr, int32_t* src, int32_t* eid,
                          int32_t* graph_off, void* stream);

/* Experiment knobs of the launchers (kernel-lab sweeps; not needed for normal use; process-wide,
 * not thread-safe).  Returns hipErrorInvalidValue for an unknown name or a value out of range;
 * "reset" restores every default.  Geometry: "fwd_lo"/"fwd_hi"/"fwd_cap", "fwd_regular_*",
 * "bwd_fused_*", "bwd_regular_*"; kernel choice: "bwd_regular_mfma" (1, default: the matrix-core
 * backward for MRP_GRAPH_REGULAR graphs of 9..16 nodes), "bwd_complete_mfma" (1, default: the
 * matrix-core backward for complete graphs of 9..16 nodes too; those of <= 8 always run the VALU
 * one), "bwd_mfma_cpw" (channel blocks per wave of the matrix-core backward, 1 or 2), "bwd_pre2" (0
 * off, 1 on, 2 on unless a grad_x base is given), "fwd_regular_split" (0, default: whole planes).
 * Knobs that name a kernel accept only the kernels the library builds: "edge_split_v"
 * (mrp_edge_encoder_fwd_split: -1, default: per shape; 1 / 3: the hidden layer shared by a workgroup
 * of 4 / 8 waves); "gemm_split" (split-bf16 compress forward / data gradient: -1 per shape (7 where
 * M % 256 == 0, else 2), 2 = 128 rows / 4 waves on 32x32x16 MFMAs, 7 = 256 rows / 8 waves on 16x16x32
 * MFMAs); "split_nt" (split-bf16 weight gradient of mrp_compress_bwd_weight_split and
 * mrp_edge_encoder_bwd_split: -1 per shape, 3 = both operands split in the kernel on 16x16x32 MFMAs,
 * 4 = the compress weight gradient with dy split once (split_rows + gemm_nt_psa; the default where
 * C >= 1024)).  Round 4's other kernel forms are lab code (tools/lab_*.hip) since ABI 18.  Tile order
 * of the split-bf16 GEMMs: "gemm_group" (runs of this many 256-row tiles walked m fastest, so an XCD's
 * concurrent workgroups share row and column blocks in its L2; 4 default, 0 = all, 1..64) for the
 * forward / data gradient, "nt_group" (the same, default 0) for the weight gradient; "enc_bwd_psa"
 * (mrp_edge_encoder_bwd_fused given w2T_packed: 2 default = both products read their A operand
 * pre-split, dz^T written as a packed image; 1 = only W2^T's image; 0 = both split in the kernel);
 * "enc_s1" / "enc_s2" (its two products' split-K counts, 0 = the planner's). */
int mrp_tuning_set(const char* name, int32_t value);

/* Library identification: ABI version (incremented on signature changes; 21 = this header: v19 plus
 * the streaming yardstick mrp_stream_copy, the device-scope stream join mrp_stream_join and the encoder's pose gradient (mrp_edge_encoder_bwd_pose
 * + workspace); 20: v19 plus a one-launch no-grad GCN layer
 * (mrp_gcn_fwd_fused), measured slower than the two launches it replaced and removed in 21
 * (tools/lab_patches/r06_fused_layer.patch); 19: v18 with
 * mrp_edge_encoder_bwd_fused taking W2^T's packed image (w2T_packed); 18: v17 without
 * mrp_edge_encoder_fwd (the fp32 one-launch encoder, superseded by mrp_edge_encoder_fwd_split) and
 * with fewer tuning knobs (only those that select kernels the library builds); 17: v16 plus
 * the split-bf16 training path of the edge encoder (mrp_edge_encoder_fwd_split_train, _bwd_prep,
 * _bwd_split, _bwd_t and their workspaces); 16: v15 plus
 * the split-bf16 weight gradient (mrp_compress_bwd_weight_split + workspace); 15: v14 plus
 * the split-bf16 compress forward / data gradient and their weight packing (mrp_compress_split_*,
 * mrp_compress_fwd_split, mrp_compress_bwd_data_split); 14: v13 plus
 * the split-bf16 edge encoder forward and its weight packing (mrp_edge_encoder_pack_bytes /
 * _pack / _fwd_split); 13: the
 * aggregation and epilogue entry points of v10, the matrix-core compress forward and gradients,
 * mrp_compress_fwd / _bwd_data / _bwd_weight of v12 (v11's forward-only fused and two-source
 * compress kernels, their weight packing and mrp_film_gate are gone), and the edge encoder's
 * second Linear and whole forward, mrp_edge_logits_fwd / mrp_edge_encoder_fwd). */
int mrp_abi_version(void);

/* The streaming yardstick the benchmark reports beside every aggregation roofline (ceiling_frac):
 * dst = src over `bytes` (a multiple of 16; 16-byte aligned pointers) as one nontemporal 16-byte load
 * and store per thread — the 1-read-1-write copy the HBM-bound kernels are measured against on the
 * same box in the same run.  Not part of the GCN path. */
int mrp_stream_copy(const void* src, void* dst, int64_t bytes, void* stream);

/* Stream join: work enqueued on `waiter` after this call waits for everything enqueued on `signaller`
 * before it — an event recorded with a device-scope release (no system-scope cache writeback: the
 * joined work is on the same device) that `waiter` waits on.  The inference encoder's stream joins the
 * caller's stream with it (encoder.py).  Returns a hipError_t. */
int mrp_stream_join(void* waiter, void* signaller);

/* Human-readable text for a return code (static storage). */
const char* mrp_error_string(int code);

#ifdef __cplusplus
}
#endif

#endif /* MRP_GNN_H */
