// Python bindings for the gfx950 kernels (module llmss_amd._C).
//
// Pointers and the HIP stream are passed as integers: the Python layer (llmss_amd/ops/hip.py)
// owns tensor validation (dtype, contiguity, shapes vs. the grid each kernel assumes) so that a
// malformed call raises in Python instead of faulting the GPU. No torch headers are needed, which
// keeps the build a plain hipcc compile (no hipify step, no CUDA-compat layer).
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <stdint.h>

namespace py = pybind11;

void launch_add_norm(const void* x, int64_t x_stride, const void* res_in, void* res_out, const void* w, const void* b,
                     void* y, int64_t y_stride, int T, int H, float eps, bool rms, hipStream_t st, void* q8,
                     void* s8, int xcw);
void launch_embed(const void* ids, const void* pos, const void* wte, const void* wpe, void* out, int T, int H,
                  int vocab, hipStream_t st);
void launch_rope_cache(void* qkv, int64_t row_stride, const void* pos, const void* cos_t, const void* sin_t, void* kc,
                       void* vc, const void* slot, int T, int nh, int nkv, int D, int rot, int block_size, int k_off,
                       int v_off, int style, bool do_rope, const void* part, int S, int64_t slab, const void* bias,
                       hipStream_t st, bool kv8);
void launch_attn_decode(const void* q, int64_t q_stride, const void* kc, const void* vc, const void* block_tables,
                        int bt_stride, const void* ctx_lens, void* out, int64_t out_stride, void* part_o,
                        void* part_ml, int B, int nh, int nkv, int D, int block_size, int nsplit, int part_size,
                        float scale, hipStream_t st, bool kv8);
void launch_attn_prefill(const void* qkv, int64_t row_stride, int T, const void* cu_seqlens, void* out,
                         int64_t out_stride, int B, int max_seqlen, int nh, int nkv, int D, int k_off, int v_off,
                         float scale, hipStream_t st);
void attn_prefill_set_version(int v);
void attn_prefill_set_waves(int nw);
void gemm_big_set_group(int g);
void launch_cand_topk(const void* logits, int64_t ld, int B, int vl, int lo, int V, const void* temperature,
                      const void* top_k, int K, int KC, void* pack, int64_t ldp, hipStream_t st, int shards);
void launch_sample_cand(const void* pack, int64_t ldp, int B, int groups, int KC, const void* temperature,
                        const void* top_k, const void* top_p, const void* seeds, void* out, void* out2, hipStream_t st);
void launch_ce_loss(const void* logits, int64_t ld, bool fp32, const void* labels, int T, int V, void* loss,
                    hipStream_t st);
void launch_attn_extend(const void* q, int64_t q_stride, const void* k_cache, const void* v_cache,
                        const void* block_tables, int max_blocks, const void* cu_q, const void* ctx_lens, void* out,
                        int64_t out_stride, int B, int max_qlen, int nh, int nkv, int D, int bs, float scale,
                        hipStream_t st, bool kv8, void* q8, void* s8);
int launch_gemm_qkv_args(const void* x, int64_t ldx, const void* w, int64_t ldw, const void* bias, void* y, int64_t ldy,
                         int M, int N, int K, void* workspace, int64_t ws_bytes, int nt_hint, int split_hint,
                         const void* pos, const void* cos_t, const void* sin_t, void* kc, void* vc, const void* slot,
                         int nh, int nkv, int D, int rot, int block_size, int style, bool do_rope, hipStream_t st);
int launch_gemm(const void* x, int64_t ldx, const void* w, int64_t ldw, bool w_fp8, const void* w_scale,
                const void* bias, void* y, int64_t ldy, int M, int N, int K, int act, bool glu, void* workspace,
                int64_t ws_bytes, int nt_hint, int split_hint, bool partial_out, hipStream_t st);
void gemm_plan(int M, int N, int K, bool w_fp8, int* nt, int* splitk);
void gemm_tuned_set(int M, int N, int K, bool glu, int kind, int nt_hint, int split);
void gemm_tuned_clear();
void gemm_reserve_streamk(int n);
void gemm_set_slot(int s);
int launch_gemm_f8f8(const void* xq, int64_t ldx, const void* xs, const void* wq, int64_t ldw, const void* wsc,
                     const void* bias, void* y, int64_t ldy, int M, int N, int K, int act, bool glu, int tile,
                     int depth, int split, void* workspace, int64_t ws_bytes, hipStream_t st, bool partial_out,
                     bool ilv, void* mxq, void* mxs, const void* asc);
int gemm_f8f8_partial_slabs(int M, int N, int K, bool glu, int act, int tile, int split, int64_t ws_bytes);
int gemm_partial_slabs(int M, int N, int K, bool w_fp8, bool glu, int act, int nt_hint, int split_hint,
                       int64_t ws_bytes);
void attn_decode_set_unroll(int u);
void launch_comm_model(void* buf, int channels, int64_t nbytes, double us, hipStream_t st);
int64_t comm_model_slice(int channels, int64_t nbytes);

bool gemm_tuned_get(int M, int N, int K, bool glu, int kind, int* nt_hint, int* split);
void launch_add_norm_partial(const void* part, int S, int64_t slab, const void* xbias, const void* res_in,
                             void* res_out, const void* w, const void* b, void* y, int64_t y_stride, int T, int H,
                             float eps, bool rms, hipStream_t st, void* q8, void* s8);
void launch_sample(const void* logits, int64_t ld, bool fp32_logits, int B, int V, const void* temperature,
                   const void* top_k, const void* top_p, const void* seeds, void* out, void* out2, hipStream_t st);
void launch_quant_fp8_rows(const void* w, void* q, void* scale, int64_t N, int64_t K, hipStream_t st);
void launch_quant_fp8_rows_ld(const void* x, int64_t ldx, void* q, void* scale, int64_t M, int64_t K, hipStream_t st);
void launch_dequant_fp8_rows(const void* q, const void* scale, void* w, int64_t N, int64_t K, hipStream_t st);

void register_runtime(py::module_& m);  // host-side C++ runtime (runtime.cpp)
void register_comm(py::module_& m);     // RCCL communicator (comm.cpp)
void register_ctrl(py::module_& m);     // shared-memory control ring (ctrl.cpp)

#define P(x) reinterpret_cast<void*>(static_cast<uintptr_t>(x))
#define CP(x) reinterpret_cast<const void*>(static_cast<uintptr_t>(x))
#define S(x) reinterpret_cast<hipStream_t>(static_cast<uintptr_t>(x))

PYBIND11_MODULE(_C, m) {
  m.doc() = "llmss_amd gfx950 HIP kernels + native runtime";
  m.def("add_norm", [](uintptr_t x, int64_t xs, uintptr_t ri, uintptr_t ro, uintptr_t w, uintptr_t b, uintptr_t y,
                       int64_t ys, int T, int H, float eps, bool rms, uintptr_t st, uintptr_t q8, uintptr_t s8, int xcw) {
    launch_add_norm(CP(x), xs, CP(ri), P(ro), CP(w), CP(b), P(y), ys, T, H, eps, rms, S(st), P(q8), P(s8), xcw);
  }, pybind11::arg("x"), pybind11::arg("xs"), pybind11::arg("ri"), pybind11::arg("ro"), pybind11::arg("w"),
     pybind11::arg("b"), pybind11::arg("y"), pybind11::arg("ys"), pybind11::arg("T"), pybind11::arg("H"),
     pybind11::arg("eps"), pybind11::arg("rms"), pybind11::arg("st"), pybind11::arg("q8") = 0,
     pybind11::arg("s8") = 0, pybind11::arg("xcw") = 0);
  m.def("embed", [](uintptr_t ids, uintptr_t pos, uintptr_t wte, uintptr_t wpe, uintptr_t out, int T, int H, int V,
                    uintptr_t st) { launch_embed(CP(ids), CP(pos), CP(wte), CP(wpe), P(out), T, H, V, S(st)); });
  m.def("rope_cache", [](uintptr_t qkv, int64_t rs, uintptr_t pos, uintptr_t cos_t, uintptr_t sin_t, uintptr_t kc,
                         uintptr_t vc, uintptr_t slot, int T, int nh, int nkv, int D, int rot, int bs, int k_off,
                         int v_off, int style, bool do_rope, uintptr_t part, int nslab, int64_t slab, uintptr_t bias,
                         uintptr_t st, bool kv8) {
    launch_rope_cache(P(qkv), rs, CP(pos), CP(cos_t), CP(sin_t), P(kc), P(vc), CP(slot), T, nh, nkv, D, rot, bs, k_off,
                      v_off, style, do_rope, CP(part), nslab, slab, CP(bias), S(st), kv8);
  });
  m.def("attn_decode", [](uintptr_t q, int64_t qs, uintptr_t kc, uintptr_t vc, uintptr_t bt, int bts, uintptr_t cl,
                          uintptr_t out, int64_t os, uintptr_t po, uintptr_t pml, int B, int nh, int nkv, int D, int bs,
                          int nsplit, int psize, float scale, uintptr_t st, bool kv8) {
    launch_attn_decode(CP(q), qs, CP(kc), CP(vc), CP(bt), bts, CP(cl), P(out), os, P(po), P(pml), B, nh, nkv, D, bs,
                       nsplit, psize, scale, S(st), kv8);
  });
  m.def("attn_prefill", [](uintptr_t qkv, int64_t rs, int T, uintptr_t cu, uintptr_t out, int64_t os, int B,
                           int maxlen, int nh, int nkv, int D, int k_off, int v_off, float scale, uintptr_t st) {
    launch_attn_prefill(CP(qkv), rs, T, CP(cu), P(out), os, B, maxlen, nh, nkv, D, k_off, v_off, scale, S(st));
  });
  m.def("attn_prefill_set_version", &attn_prefill_set_version);
  m.def("attn_prefill_set_waves", &attn_prefill_set_waves);
  m.def("gemm_big_set_group", &gemm_big_set_group);
  m.def("cand_topk", [](uintptr_t lg, int64_t ld, int B, int vl, int lo, int V, uintptr_t temp, uintptr_t topk, int K,
                        int KC, uintptr_t pack, int64_t ldp, uintptr_t st, int shards) {
    launch_cand_topk(CP(lg), ld, B, vl, lo, V, CP(temp), CP(topk), K, KC, P(pack), ldp, S(st), shards);
  }, pybind11::arg("lg"), pybind11::arg("ld"), pybind11::arg("B"), pybind11::arg("vl"), pybind11::arg("lo"),
     pybind11::arg("V"), pybind11::arg("temp"), pybind11::arg("topk"), pybind11::arg("K"), pybind11::arg("KC"),
     pybind11::arg("pack"), pybind11::arg("ldp"), pybind11::arg("st"), pybind11::arg("shards") = 1);
  m.def("sample_cand", [](uintptr_t pack, int64_t ldp, int B, int groups, int KC, uintptr_t temp, uintptr_t topk,
                          uintptr_t topp, uintptr_t seeds, uintptr_t out, uintptr_t out2, uintptr_t st) {
    launch_sample_cand(CP(pack), ldp, B, groups, KC, CP(temp), CP(topk), CP(topp), CP(seeds), P(out), P(out2), S(st));
  });
  m.def("ce_loss", [](uintptr_t lg, int64_t ld, bool fp32, uintptr_t lab, int T, int V, uintptr_t loss, uintptr_t st) {
    launch_ce_loss(CP(lg), ld, fp32, CP(lab), T, V, P(loss), S(st));
  });
  m.def("attn_extend", [](uintptr_t q, int64_t qs, uintptr_t kc, uintptr_t vc, uintptr_t bt, int maxb, uintptr_t cu,
                          uintptr_t cl, uintptr_t out, int64_t os, int B, int maxq, int nh, int nkv, int D, int bs,
                          float scale, uintptr_t st, bool kv8, uintptr_t q8, uintptr_t s8) {
    launch_attn_extend(CP(q), qs, CP(kc), CP(vc), CP(bt), maxb, CP(cu), CP(cl), P(out), os, B, maxq, nh, nkv, D, bs,
                       scale, S(st), kv8, P(q8), P(s8));
  }, pybind11::arg("q"), pybind11::arg("qs"), pybind11::arg("kc"), pybind11::arg("vc"), pybind11::arg("bt"),
     pybind11::arg("maxb"), pybind11::arg("cu"), pybind11::arg("cl"), pybind11::arg("out"), pybind11::arg("os"),
     pybind11::arg("B"), pybind11::arg("maxq"), pybind11::arg("nh"), pybind11::arg("nkv"), pybind11::arg("D"),
     pybind11::arg("bs"), pybind11::arg("scale"), pybind11::arg("st"), pybind11::arg("kv8"), pybind11::arg("q8") = 0,
     pybind11::arg("s8") = 0);
  m.def("gemm", [](uintptr_t x, int64_t ldx, uintptr_t w, int64_t ldw, bool fp8, uintptr_t ws, uintptr_t bias,
                   uintptr_t y, int64_t ldy, int M, int N, int K, int act, bool glu, uintptr_t work, int64_t wbytes,
                   int nt_hint, int split_hint, bool partial_out, uintptr_t st) {
    return launch_gemm(CP(x), ldx, CP(w), ldw, fp8, CP(ws), CP(bias), P(y), ldy, M, N, K, act, glu, P(work), wbytes,
                       nt_hint, split_hint, partial_out, S(st));
  });
  m.def("gemm_qkv", [](uintptr_t x, int64_t ldx, uintptr_t w, int64_t ldw, uintptr_t bias, uintptr_t y, int64_t ldy,
                       int M, int N, int K, uintptr_t work, int64_t wbytes, int nt_hint, int split_hint, uintptr_t pos,
                       uintptr_t cos_t, uintptr_t sin_t, uintptr_t kc, uintptr_t vc, uintptr_t slot, int nh, int nkv,
                       int D, int rot, int bs, int style, bool do_rope, uintptr_t st) {
    return launch_gemm_qkv_args(CP(x), ldx, CP(w), ldw, CP(bias), P(y), ldy, M, N, K, P(work), wbytes, nt_hint,
                                split_hint, CP(pos), CP(cos_t), CP(sin_t), P(kc), P(vc), CP(slot), nh, nkv, D, rot, bs,
                                style, do_rope, S(st));
  }, pybind11::arg("x"), pybind11::arg("ldx"), pybind11::arg("w"), pybind11::arg("ldw"), pybind11::arg("bias"),
     pybind11::arg("y"), pybind11::arg("ldy"), pybind11::arg("M"), pybind11::arg("N"), pybind11::arg("K"),
     pybind11::arg("work"), pybind11::arg("wbytes"), pybind11::arg("nt_hint"), pybind11::arg("split_hint"),
     pybind11::arg("pos"), pybind11::arg("cos_t"), pybind11::arg("sin_t"), pybind11::arg("kc"), pybind11::arg("vc"),
     pybind11::arg("slot"), pybind11::arg("nh"), pybind11::arg("nkv"), pybind11::arg("D"), pybind11::arg("rot"),
     pybind11::arg("bs"), pybind11::arg("style"), pybind11::arg("do_rope"), pybind11::arg("st"));
  m.def("gemm_plan", [](int M, int N, int K, bool fp8) {
    int nt, s;
    gemm_plan(M, N, K, fp8, &nt, &s);
    return py::make_tuple(nt, s);
  });
  m.def("gemm_tuned_set", &gemm_tuned_set);
  m.def("gemm_tuned_clear", &gemm_tuned_clear);
  m.def("gemm_reserve_streamk", &gemm_reserve_streamk);
  m.def("gemm_set_slot", &gemm_set_slot);
  m.def("gemm_f8f8", [](uintptr_t xq, int64_t ldx, uintptr_t xs, uintptr_t wq, int64_t ldw, uintptr_t wsc,
                        uintptr_t bias, uintptr_t y, int64_t ldy, int M, int N, int K, int act, bool glu, int tile,
                        int depth, int split, uintptr_t work, int64_t wbytes, uintptr_t st, bool partial_out, bool ilv,
                        uintptr_t mxq, uintptr_t mxs, uintptr_t asc) {
    return launch_gemm_f8f8(CP(xq), ldx, CP(xs), CP(wq), ldw, CP(wsc), CP(bias), P(y), ldy, M, N, K, act, glu, tile,
                            depth, split, P(work), wbytes, S(st), partial_out, ilv, P(mxq), P(mxs), CP(asc));
  }, pybind11::arg("xq"), pybind11::arg("ldx"), pybind11::arg("xs"), pybind11::arg("wq"), pybind11::arg("ldw"),
     pybind11::arg("wsc"), pybind11::arg("bias"), pybind11::arg("y"), pybind11::arg("ldy"), pybind11::arg("M"),
     pybind11::arg("N"), pybind11::arg("K"), pybind11::arg("act"), pybind11::arg("glu"), pybind11::arg("tile"),
     pybind11::arg("depth"), pybind11::arg("split"), pybind11::arg("work"), pybind11::arg("wbytes"),
     pybind11::arg("st"), pybind11::arg("partial_out") = false, pybind11::arg("ilv") = false,
     pybind11::arg("mxq") = 0, pybind11::arg("mxs") = 0, pybind11::arg("asc") = 0);
  m.def("gemm_f8f8_partial_slabs", &gemm_f8f8_partial_slabs);
  m.def("gemm_partial_slabs", &gemm_partial_slabs);
  m.def("attn_decode_set_unroll", &attn_decode_set_unroll);
  m.def("comm_model", [](uintptr_t buf, int channels, int64_t nbytes, double us, uintptr_t st) {
    launch_comm_model(P(buf), channels, nbytes, us, S(st));
  });
  m.def("comm_model_slice", &comm_model_slice);
  m.def("gemm_tuned_get", [](int M, int N, int K, bool glu, int kind) -> py::object {
    int nt, s;
    if (!gemm_tuned_get(M, N, K, glu, kind, &nt, &s)) return py::none();
    return py::make_tuple(nt, s);
  });
  m.def("add_norm_partial", [](uintptr_t part, int S, int64_t slab, uintptr_t xbias, uintptr_t ri, uintptr_t ro,
                               uintptr_t w, uintptr_t b, uintptr_t y, int64_t ys, int T, int H, float eps, bool rms,
                               uintptr_t st, uintptr_t q8, uintptr_t s8) {
    launch_add_norm_partial(CP(part), S, slab, CP(xbias), CP(ri), P(ro), CP(w), CP(b), P(y), ys, T, H, eps, rms, S(st),
                            P(q8), P(s8));
  }, pybind11::arg("part"), pybind11::arg("S"), pybind11::arg("slab"), pybind11::arg("xbias"), pybind11::arg("ri"),
     pybind11::arg("ro"), pybind11::arg("w"), pybind11::arg("b"), pybind11::arg("y"), pybind11::arg("ys"),
     pybind11::arg("T"), pybind11::arg("H"), pybind11::arg("eps"), pybind11::arg("rms"), pybind11::arg("st"),
     pybind11::arg("q8") = 0, pybind11::arg("s8") = 0);
  m.def("sample", [](uintptr_t logits, int64_t ld, bool fp32, int B, int V, uintptr_t temp, uintptr_t topk,
                     uintptr_t topp, uintptr_t seeds, uintptr_t out, uintptr_t out2, uintptr_t st) {
    launch_sample(CP(logits), ld, fp32, B, V, CP(temp), CP(topk), CP(topp), CP(seeds), P(out), P(out2), S(st));
  });
  m.def("quant_fp8_rows", [](uintptr_t w, uintptr_t q, uintptr_t scale, int64_t N, int64_t K, uintptr_t st) {
    launch_quant_fp8_rows(CP(w), P(q), P(scale), N, K, S(st));
  });
  m.def("quant_fp8_rows_ld", [](uintptr_t x, int64_t ldx, uintptr_t q, uintptr_t scale, int64_t M, int64_t K,
                                uintptr_t st) { launch_quant_fp8_rows_ld(CP(x), ldx, P(q), P(scale), M, K, S(st)); });
  m.def("dequant_fp8_rows", [](uintptr_t q, uintptr_t scale, uintptr_t w, int64_t N, int64_t K, uintptr_t st) {
    launch_dequant_fp8_rows(CP(q), CP(scale), P(w), N, K, S(st));
  });
  register_runtime(m);
  register_comm(m);
  register_ctrl(m);
}
