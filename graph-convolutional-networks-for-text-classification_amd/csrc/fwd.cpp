// Whole-forward launch record (gcnk_gcn_forward_f32, include/gcnk.h).
//
// GCN.forward (reference layer.py:164-190) is called eagerly once or twice per
// epoch by the trainer (trainer.py:357 train, trainer.py:382 eval).  Issued op
// by op from Python, each of its 4-5 launches pays argument marshalling, plan
// and workspace lookups and device guards (the eager forward took 76-92 us
// for 26 us of kernels, profiles/r03_eager_forward_host_profile.log).  Here the
// caller fills a gcnk_gcn_fwd record once with everything that is fixed per
// (graph, features, widths, stream) and a call runs the launches straight
// through the per-op entry points: the same kernels, arguments and order, so
// the outputs are bitwise those of the per-op path.
#include "gcnk_common.h"

using namespace gcnk;

namespace {

int spmm_ref(const gcnk_plan_ref& p, const float* B, int64_t ldb, int32_t F, float* C, int64_t ldc, const float* bias,
             int32_t epi, const uint8_t* mask, int64_t ldm, float scale, float keep, uint64_t seed, uint64_t offset,
             const uint64_t* rng_base, void* stream) {
  return gcnk_spmm_csr_f32(p.plan, p.hdr, B, ldb, F, C, ldc, bias, epi, mask, ldm, scale, keep, seed, offset, rng_base,
                           p.workspace, p.workspace_bytes, p.counters, p.counter_bytes, p.lanes_hint, stream);
}

// S1 = X W1 (sparse X through its plan, dense X on the MFMA GEMM)
int first_product(const gcnk_gcn_fwd& r, const float* W1, void* stream) {
  if (r.x.plan)
    return spmm_ref(r.x, W1, r.F, r.F, r.s1, r.lds1, nullptr, GCNK_EPI_NONE, nullptr, 0, 1.f, 1.f, 0, 0, nullptr,
                    stream);
  return gcnk_gemm_f32(0, 0, r.x_rows, r.F, r.x_cols, r.x_dense, r.ldx, W1, r.F, r.s1, r.lds1, nullptr,
                       GCNK_GEMM_EPI_NONE, nullptr, 0, 1.f, r.x_split_k, r.gemm_ws, r.gemm_ws_bytes, stream);
}

}  // namespace

extern "C" int gcnk_gcn_forward_f32(const gcnk_gcn_fwd* rec, const float* W1, const float* b1, const float* W2,
                                    const float* b2, float* out, int64_t ldo, float* H1, int64_t ldh,
                                    int32_t epilogue, const uint8_t* drop_mask, int64_t ldm, float drop_scale,
                                    float keep_prob, uint64_t seed, uint64_t offset, const uint64_t* rng_base,
                                    void* stream) {
  if (!rec || !W1 || !W2 || !out || (rec->kind != GCNK_FWD_DENSE_AX && !rec->s1) || !rec->s2 || !rec->aP.plan ||
      rec->M <= 0 || rec->F <= 0 ||
      rec->P <= 0 || ldo < rec->P || (H1 && ldh < rec->F)) {
    set_error("gcnk_gcn_forward_f32: null record/operand or bad sizes");
    return GCNK_EARG;
  }
  const gcnk_gcn_fwd& r = *rec;
  if ((r.kind == GCNK_FWD_FACTORED && (!r.U || !r.rec)) || (r.kind == GCNK_FWD_DENSE_AX && !r.U) ||
      ((r.kind == GCNK_FWD_SPMM_PROJ || r.kind == GCNK_FWD_SPMM_GEMM) && !r.aF.plan) ||
      (r.kind == GCNK_FWD_SPMM_GEMM && !H1 && !r.h1_tmp) ||
      (r.kind != GCNK_FWD_DENSE_AX && !r.x.plan && !r.x_dense)) {
    set_error("gcnk_gcn_forward_f32: record kind %d is missing an operand (U / records / F-wide plan / H1 scratch / X)",
              r.kind);
    return GCNK_EARG;
  }
  int rc = GCNK_OK;
  switch (r.kind) {
    case GCNK_FWD_FACTORED:
      if ((rc = first_product(r, W1, stream)) != GCNK_OK) return rc;
      rc = gcnk_hubfactor_gc1_f32(r.M, r.F, r.Kc, r.nhub, r.P, r.U, r.ldu, W1, r.F, r.k0, r.s1, r.lds1, r.rec,
                                  r.rec_words, b1, epilogue, drop_mask, ldm, drop_scale, keep_prob, seed, offset,
                                  rng_base, W2, r.P, H1, ldh, r.s2, r.lds2, stream);
      break;
    case GCNK_FWD_DENSE_AX:
      rc = gcnk_dense_gc1_f32(r.M, r.Kc, r.F, r.P, r.U, r.ldu, W1, r.F, b1, epilogue, drop_mask, ldm, drop_scale,
                              keep_prob, seed, offset, rng_base, W2, r.P, H1, ldh, r.s2, r.lds2, stream);
      break;
    case GCNK_FWD_SPMM_PROJ:
      if ((rc = first_product(r, W1, stream)) != GCNK_OK) return rc;
      rc = gcnk_spmm_proj_f32(r.aF.plan, r.aF.hdr, r.s1, r.lds1, r.F, H1, ldh, b1, epilogue, drop_mask, ldm, drop_scale,
                              keep_prob, seed, offset, rng_base, W2, r.P, r.P, r.s2, r.lds2, r.aF.workspace,
                              r.aF.workspace_bytes, r.aF.counters, r.aF.counter_bytes, r.aF.lanes_hint, stream);
      // outside the fused kernel's range (width, alignment of an operand): the
      // same result from the SpMM into H1 (or the record's scratch) + the GEMM,
      // as ops.spmm_proj does (nothing was launched by the refused call)
      if (rc != GCNK_EUNSUP || (!H1 && !r.h1_tmp)) break;
      [[fallthrough]];
    case GCNK_FWD_SPMM_GEMM: {
      float* h = H1 ? H1 : r.h1_tmp;
      const int64_t lh = H1 ? ldh : r.ld_h1_tmp;
      if (r.kind == GCNK_FWD_SPMM_GEMM && (rc = first_product(r, W1, stream)) != GCNK_OK) return rc;
      if ((rc = spmm_ref(r.aF, r.s1, r.lds1, r.F, h, lh, b1, epilogue, drop_mask, ldm, drop_scale, keep_prob, seed,
                         offset, rng_base, stream)) != GCNK_OK)
        return rc;
      rc = gcnk_gemm_f32(0, 0, r.M, r.P, r.F, h, lh, W2, r.P, r.s2, r.lds2, nullptr, GCNK_GEMM_EPI_NONE, nullptr, 0,
                         1.f, 1, r.gemm_ws, r.gemm_ws_bytes, stream);
      break;
    }
    default:
      set_error("gcnk_gcn_forward_f32: unknown record kind %d", r.kind);
      return GCNK_EARG;
  }
  if (rc != GCNK_OK) return rc;
  // gc2: logits = A-hat S2 + b2  (layer.py:106,110)
  return spmm_ref(r.aP, r.s2, r.lds2, r.P, out, ldo, b2, b2 ? GCNK_EPI_BIAS : GCNK_EPI_NONE, nullptr, 0, 1.f, 1.f, 0, 0,
                  nullptr, stream);
}

// Layout check for bindings that mirror the record (ctypes): sizes and offsets.
extern "C" int32_t gcnk_gcn_fwd_layout(int64_t* out, int32_t n) {
  const int64_t v[] = {(int64_t)sizeof(gcnk_plan_ref), (int64_t)sizeof(gcnk_gcn_fwd),
                       (int64_t)offsetof(gcnk_gcn_fwd, x), (int64_t)offsetof(gcnk_gcn_fwd, U),
                       (int64_t)offsetof(gcnk_gcn_fwd, aF), (int64_t)offsetof(gcnk_gcn_fwd, aP),
                       (int64_t)offsetof(gcnk_gcn_fwd, ld_h1_tmp), (int64_t)offsetof(gcnk_plan_ref, lanes_hint),
                       (int64_t)sizeof(gcnk_gcn_bwd), (int64_t)offsetof(gcnk_gcn_bwd, xT),
                       (int64_t)offsetof(gcnk_gcn_bwd, bwd2_ws_bytes)};
  const int32_t m = (int32_t)(sizeof(v) / sizeof(v[0]));
  for (int32_t i = 0; i < n && i < m; ++i) out[i] = v[i];
  return m;
}

// The backward record (gcnk_gcn_backward_f32): ops.GCNFn.backward's launches.
extern "C" int gcnk_gcn_backward_f32(const gcnk_gcn_bwd* rec, const float* G, const float* H1, int64_t ldh,
                                     const float* W2, float scale, float* gW1, float* gb1, float* gW2, float* gb2,
                                     void* stream) {
  const bool ax = (rec && (rec->flags & GCNK_BWD_AX_DIRECT));
  if (!rec || !G || !H1 || !W2 || rec->M <= 0 || rec->F <= 0 || rec->P <= 0 || ldh < rec->F || !rec->aTP.plan ||
      !rec->gS2 || !rec->gZ1 ||
      (gW1 && (ax ? !rec->x_dense : (!rec->aTF.plan || !rec->gS1 || (!rec->xT.plan && !rec->x_dense))))) {
    set_error("gcnk_gcn_backward_f32: null record/operand or incomplete record");
    return GCNK_EARG;
  }
  const gcnk_gcn_bwd& r = *rec;
  int rc;
  // gS2 = A-hat^T G  (autograd of layer.py:106 in gc2)
  if ((rc = spmm_ref(r.aTP, G, r.P, r.P, r.gS2, r.P, nullptr, GCNK_EPI_NONE, nullptr, 0, 1.f, 1.f, 0, 0, nullptr,
                     stream)) != GCNK_OK)
    return rc;
  // gc2's weight/bias grads and gc1's ReLU + dropout backward (layer.py:102-110,182-188); the fixed-order
  // sum of its gW2 / gb1 / gb2 partials has no consumer before Adam, so it rides in the backward's last
  // launch (X^T gS1's tile reduce) when that launch exists, else it runs at the end as its own
  SideReduce side;
  if ((rc = gcn_bwd2_main(H1, ldh, r.gS2, r.P, W2, r.P, gb2 ? G : nullptr, r.P, r.M, r.F, r.P, scale, r.gZ1, r.F,
                          gW2, gb1, gb2, r.bwd2_ws, r.bwd2_ws_bytes, stream, &side)) != GCNK_OK)
    return rc;
  if (!gW1) return side_reduce_launch(side, stream);
  if (ax) {  // gW1 = (A-hat X)^T gZ1: the DENSE_AX forward's Z1 = (A-hat X) W1
    if ((rc = gcnk_gemm_f32(1, 0, r.x_cols, r.F, r.x_rows, r.x_dense, r.ldx, r.gZ1, r.F, gW1, r.F, nullptr,
                            GCNK_GEMM_EPI_NONE, nullptr, 0, 1.f, r.x_split_k, r.gemm_ws, r.gemm_ws_bytes, stream)) !=
        GCNK_OK)
      return rc;
    return side_reduce_launch(side, stream);
  }
  // gS1 = A-hat^T gZ1, gW1 = X^T gS1  (autograd of layer.py:106, :102 in gc1)
  if ((rc = spmm_ref(r.aTF, r.gZ1, r.F, r.F, r.gS1, r.F, nullptr, GCNK_EPI_NONE, nullptr, 0, 1.f, 1.f, 0, 0, nullptr,
                     stream)) != GCNK_OK)
    return rc;
  int carried = 0;
  if (r.xT.plan)
    rc = spmm_csr_f32_side(r.xT.plan, r.xT.hdr, r.gS1, r.F, r.F, gW1, r.F, r.xT.workspace, r.xT.workspace_bytes,
                           r.xT.counters, r.xT.counter_bytes, r.xT.lanes_hint, stream, side, &carried);
  else
    rc = gcnk_gemm_f32(1, 0, r.x_cols, r.F, r.x_rows, r.x_dense, r.ldx, r.gS1, r.F, gW1, r.F, nullptr,
                       GCNK_GEMM_EPI_NONE, nullptr, 0, 1.f, r.x_split_k, r.gemm_ws, r.gemm_ws_bytes, stream);
  if (rc != GCNK_OK || carried) return rc;
  return side_reduce_launch(side, stream);
}
