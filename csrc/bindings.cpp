// pybind11 bindings of the fluxmpi_amd native library -> module `fluxmpi_amd._C`.
//
// Pointers and streams cross the boundary as integers (tensor.data_ptr(),
// torch.cuda.Stream.cuda_stream), which keeps this module independent of the
// ATen C++ ABI and lets it launch on any stream, including during HIP-graph
// capture.
#include <array>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "api.h"
#include "comm/rccl_comm.h"

namespace py = pybind11;
using namespace fluxmpi;

static hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

PYBIND11_MODULE(_C, m) {
  m.doc() = "fluxmpi_amd native library: gfx950 HIP kernels + RCCL communicator";

  m.def("mt_copy",
        [](const std::vector<uintptr_t>& src, const std::vector<uintptr_t>& dst, const std::vector<int64_t>& numel,
           int in_dtype, int out_dtype, float scale, uintptr_t stream) {
          mt_copy(src, dst, numel, in_dtype, out_dtype, scale, S(stream));
        },
        py::arg("src"), py::arg("dst"), py::arg("numel"), py::arg("in_dtype"), py::arg("out_dtype"),
        py::arg("scale"), py::arg("stream"));
  m.def("mt_fill",
        [](const std::vector<uintptr_t>& dst, const std::vector<int64_t>& numel, int dtype, float value,
           uintptr_t stream) { mt_fill(dst, numel, dtype, value, S(stream)); });
  m.def("mt_sumsq",
        [](const std::vector<uintptr_t>& src, const std::vector<int64_t>& numel, int dtype, uintptr_t out,
           uintptr_t stream) { mt_sumsq(src, numel, dtype, reinterpret_cast<float*>(out), S(stream)); });

  m.def("mt_adam",
        [](const std::vector<uintptr_t>& p, const std::vector<uintptr_t>& g, const std::vector<uintptr_t>& mm,
           const std::vector<uintptr_t>& vv, const std::vector<uintptr_t>& master, const std::vector<int64_t>& numel,
           int p_dtype, int g_dtype, int s_dtype, float lr, float beta1, float beta2, float eps, float bc1,
           float bc2, float weight_decay, float grad_scale, uintptr_t dev_hyper, uintptr_t dev_gscale,
           uintptr_t stream) {
          AdamHyper h{lr, beta1, beta2, eps, bc1, bc2, weight_decay, grad_scale,
                      reinterpret_cast<const float*>(dev_hyper), reinterpret_cast<const float*>(dev_gscale)};
          mt_adam(p, g, mm, vv, master, numel, p_dtype, g_dtype, s_dtype, h, S(stream));
        },
        py::arg("param"), py::arg("grad"), py::arg("m"), py::arg("v"), py::arg("master"), py::arg("numel"),
        py::arg("p_dtype"), py::arg("g_dtype"), py::arg("s_dtype"), py::arg("lr"), py::arg("beta1"),
        py::arg("beta2"), py::arg("eps"), py::arg("bc1"), py::arg("bc2"), py::arg("weight_decay"),
        py::arg("grad_scale"), py::arg("dev_hyper"), py::arg("dev_gscale"), py::arg("stream"));
  m.def("adam_advance", [](uintptr_t dev, float b1, float b2, uintptr_t stream) {
    adam_advance(reinterpret_cast<float*>(dev), b1, b2, S(stream));
  });
  m.def("mt_sgd",
        [](const std::vector<uintptr_t>& p, const std::vector<uintptr_t>& g, const std::vector<uintptr_t>& buf,
           const std::vector<uintptr_t>& master, const std::vector<int64_t>& numel, int p_dtype, int g_dtype,
           int s_dtype, float lr, float momentum, float weight_decay, float grad_scale, int nesterov,
           uintptr_t dev_lr, uintptr_t stream) {
          SgdHyper h{lr, momentum, weight_decay, grad_scale, nesterov, reinterpret_cast<const float*>(dev_lr)};
          mt_sgd(p, g, buf, master, numel, p_dtype, g_dtype, s_dtype, h, S(stream));
        },
        py::arg("param"), py::arg("grad"), py::arg("buf"), py::arg("master"), py::arg("numel"),
        py::arg("p_dtype"), py::arg("g_dtype"), py::arg("s_dtype"), py::arg("lr"), py::arg("momentum"),
        py::arg("weight_decay"), py::arg("grad_scale"), py::arg("nesterov"), py::arg("dev_lr"),
        py::arg("stream"));

  // ---- fused NHWC BatchNorm ------------------------------------------------
  m.def("bn_fwd_train",
        [](uintptr_t x, uintptr_t y, uintptr_t res, uintptr_t w, uintptr_t b, uintptr_t rm, uintptr_t rv,
           uintptr_t sm, uintptr_t si, uintptr_t ws, int64_t rows, int64_t C, float momentum, float eps, int relu,
           uintptr_t mask, int dtype, uintptr_t stream, uintptr_t nbt) {
          bn_fwd_train(reinterpret_cast<const void*>(x), reinterpret_cast<void*>(y), reinterpret_cast<const void*>(res),
                       reinterpret_cast<const float*>(w), reinterpret_cast<const float*>(b),
                       reinterpret_cast<float*>(rm), reinterpret_cast<float*>(rv), reinterpret_cast<float*>(sm),
                       reinterpret_cast<float*>(si), reinterpret_cast<float*>(ws), rows, C, momentum, eps, relu,
                       reinterpret_cast<uint8_t*>(mask), dtype, S(stream), reinterpret_cast<int64_t*>(nbt));
        });
  m.def("bn_fwd_infer",
        [](uintptr_t x, uintptr_t y, uintptr_t res, uintptr_t w, uintptr_t b, uintptr_t rm, uintptr_t rv,
           int64_t rows, int64_t C, float eps, int relu, int dtype, uintptr_t stream) {
          bn_fwd_infer(reinterpret_cast<const void*>(x), reinterpret_cast<void*>(y), reinterpret_cast<const void*>(res),
                       reinterpret_cast<const float*>(w), reinterpret_cast<const float*>(b),
                       reinterpret_cast<const float*>(rm), reinterpret_cast<const float*>(rv), rows, C, eps, relu,
                       dtype, S(stream));
        });
  m.def("bn_bwd",
        [](uintptr_t dy, uintptr_t x, uintptr_t y, uintptr_t mask, uintptr_t w, uintptr_t b, uintptr_t sm, uintptr_t si,
           uintptr_t dx,
           uintptr_t dres, uintptr_t dw, uintptr_t db, uintptr_t ws, int64_t rows, int64_t C, int relu, int dtype,
           uintptr_t stream, int stats_ready) {
          bn_bwd(reinterpret_cast<const void*>(dy), reinterpret_cast<const void*>(x), reinterpret_cast<const void*>(y),
                 reinterpret_cast<const uint8_t*>(mask),
                 reinterpret_cast<const float*>(w), reinterpret_cast<const float*>(b), reinterpret_cast<const float*>(sm),
                 reinterpret_cast<const float*>(si), reinterpret_cast<void*>(dx), reinterpret_cast<void*>(dres),
                 reinterpret_cast<float*>(dw), reinterpret_cast<float*>(db), reinterpret_cast<float*>(ws), rows, C,
                 relu, dtype, S(stream), stats_ready);
        });

  m.def("bn_stats_finalize",
        [](uintptr_t x, uintptr_t w, uintptr_t b, uintptr_t rm, uintptr_t rv, uintptr_t sm, uintptr_t si,
           uintptr_t scale, uintptr_t shift, uintptr_t ws, int64_t rows, int64_t C, float momentum, float eps,
           int stats_ready, int dtype, uintptr_t stream, uintptr_t nbt) {
          bn_stats_finalize(reinterpret_cast<const void*>(x), reinterpret_cast<const float*>(w),
                            reinterpret_cast<const float*>(b), reinterpret_cast<float*>(rm),
                            reinterpret_cast<float*>(rv), reinterpret_cast<float*>(sm), reinterpret_cast<float*>(si),
                            reinterpret_cast<float*>(scale), reinterpret_cast<float*>(shift),
                            reinterpret_cast<float*>(ws), rows, C, momentum, eps, stats_ready, dtype, S(stream),
                            reinterpret_cast<int64_t*>(nbt));
        });
  m.def("bn_apply",
        [](uintptr_t x, uintptr_t y, uintptr_t res, uintptr_t w, uintptr_t b, uintptr_t sm, uintptr_t si,
           int64_t rows, int64_t C, int relu, uintptr_t mask, int dtype, uintptr_t stream) {
          bn_apply(reinterpret_cast<const void*>(x), reinterpret_cast<void*>(y), reinterpret_cast<const void*>(res),
                   reinterpret_cast<const float*>(w), reinterpret_cast<const float*>(b),
                   reinterpret_cast<const float*>(sm), reinterpret_cast<const float*>(si), rows, C, relu,
                   reinterpret_cast<uint8_t*>(mask), dtype, S(stream));
        });

  m.def("bn_apply_dual",
        [](uintptr_t x, uintptr_t x2, uintptr_t y, uintptr_t w, uintptr_t b, uintptr_t sm, uintptr_t si, uintptr_t w2,
           uintptr_t b2, uintptr_t sm2, uintptr_t si2, int64_t rows, int64_t C, uintptr_t mask, int dtype,
           uintptr_t stream) {
          auto F = [](uintptr_t p) { return reinterpret_cast<const float*>(p); };
          bn_apply_dual(reinterpret_cast<const void*>(x), reinterpret_cast<const void*>(x2), reinterpret_cast<void*>(y),
                        F(w), F(b), F(sm), F(si), F(w2), F(b2), F(sm2), F(si2), rows, C,
                        reinterpret_cast<uint8_t*>(mask), dtype, S(stream));
        });
  m.def("bn_bwd_dual",
        [](uintptr_t dy, uintptr_t mask, uintptr_t x, uintptr_t x2, uintptr_t w, uintptr_t sm, uintptr_t si,
           uintptr_t w2, uintptr_t sm2, uintptr_t si2, uintptr_t dx, uintptr_t dx2, uintptr_t dw, uintptr_t db,
           uintptr_t dw2, uintptr_t db2, uintptr_t ws, uintptr_t ws2, int64_t rows, int64_t C, int dtype,
           uintptr_t stream) {
          auto F = [](uintptr_t p) { return reinterpret_cast<const float*>(p); };
          auto W = [](uintptr_t p) { return reinterpret_cast<float*>(p); };
          bn_bwd_dual(reinterpret_cast<const void*>(dy), reinterpret_cast<const uint8_t*>(mask),
                      reinterpret_cast<const void*>(x), reinterpret_cast<const void*>(x2), F(w), F(sm), F(si), F(w2),
                      F(sm2), F(si2), reinterpret_cast<void*>(dx), reinterpret_cast<void*>(dx2), W(dw), W(db), W(dw2),
                      W(db2), W(ws), W(ws2), rows, C, dtype, S(stream));
        });

  // ---- fused stem pool -------------------------------------------------------
  m.def("bn_relu_maxpool_fwd",
        [](uintptr_t x, uintptr_t scale, uintptr_t shift, uintptr_t y, uintptr_t idx, int64_t N, int64_t H, int64_t W,
           int64_t C, int K, int S, int P, int dtype, uintptr_t stream) {
          bn_relu_maxpool_fwd(reinterpret_cast<const void*>(x), reinterpret_cast<const float*>(scale),
                              reinterpret_cast<const float*>(shift), reinterpret_cast<void*>(y),
                              reinterpret_cast<uint8_t*>(idx), N, H, W, C, K, S, P, dtype, reinterpret_cast<hipStream_t>(stream));
        });
  m.def("attn_fwd", [](uintptr_t q, uintptr_t k, uintptr_t v, uintptr_t o, uintptr_t stats, int64_t sq_b,
                       int64_t sq_t, int64_t so_b, int64_t so_t, int64_t so_h, int B, int T, int H, int Dh,
                       float scale, uintptr_t stream) {
    attn_fwd(reinterpret_cast<const void*>(q), reinterpret_cast<const void*>(k), reinterpret_cast<const void*>(v),
             reinterpret_cast<void*>(o), reinterpret_cast<float*>(stats), sq_b, sq_t, so_b, so_t, so_h, B, T, H, Dh,
             scale, reinterpret_cast<hipStream_t>(stream));
  });
  m.def("attn_bwd", [](uintptr_t q, uintptr_t k, uintptr_t v, uintptr_t o, uintptr_t dout, uintptr_t dq,
                       uintptr_t dk, uintptr_t dv, uintptr_t stats, int64_t sq_b, int64_t sq_t, int64_t so_b,
                       int64_t so_t, int64_t so_h, int64_t sg_b, int64_t sg_t, int B, int T, int H, int Dh,
                       float scale, uintptr_t stream, uintptr_t colpart) {
    attn_bwd(reinterpret_cast<const void*>(q), reinterpret_cast<const void*>(k), reinterpret_cast<const void*>(v),
             reinterpret_cast<const void*>(o), reinterpret_cast<const void*>(dout), reinterpret_cast<void*>(dq),
             reinterpret_cast<void*>(dk), reinterpret_cast<void*>(dv), reinterpret_cast<float*>(stats), sq_b, sq_t,
             so_b, so_t, so_h, sg_b, sg_t, B, T, H, Dh, scale, reinterpret_cast<hipStream_t>(stream),
             reinterpret_cast<float*>(colpart));
  }, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("o"), py::arg("dout"), py::arg("dq"), py::arg("dk"),
     py::arg("dv"), py::arg("stats"), py::arg("sq_b"), py::arg("sq_t"), py::arg("so_b"), py::arg("so_t"),
     py::arg("so_h"), py::arg("sg_b"), py::arg("sg_t"), py::arg("B"), py::arg("T"), py::arg("H"), py::arg("Dh"),
     py::arg("scale"), py::arg("stream"), py::arg("colpart") = 0);
  m.def("attn_bwd_colpart_rows", &attn_bwd_colpart_rows);
  m.def("pad_c3_to_c4", [](uintptr_t x, uintptr_t y, int64_t npix, int dtype, uintptr_t stream) {
    pad_c3_to_c4(reinterpret_cast<const void*>(x), reinterpret_cast<void*>(y), npix, dtype,
                 reinterpret_cast<hipStream_t>(stream));
  });
  m.def("stem_fwd", [](uintptr_t x, uintptr_t wp, uintptr_t y, uintptr_t stats, int64_t n, uintptr_t stream) {
    stem_fwd(reinterpret_cast<const void*>(x), reinterpret_cast<const void*>(wp), reinterpret_cast<void*>(y),
             reinterpret_cast<float*>(stats), n, reinterpret_cast<hipStream_t>(stream));
  });
  m.def("stem_bwd_blocks", &stem_bwd_blocks);
  m.def("stem_part_floats", &stem_part_floats);
  m.def("stem_bwd", [](uintptr_t x, uintptr_t c, uintptr_t dp, uintptr_t idx, uintptr_t w, uintptr_t mean,
                       uintptr_t inv, uintptr_t part, int blocks, uintptr_t stats, uintptr_t dw_bn, uintptr_t db_bn,
                       uintptr_t dwp, int64_t n, uintptr_t stream) {
    auto F = [](uintptr_t q) { return reinterpret_cast<const float*>(q); };
    auto W = [](uintptr_t q) { return reinterpret_cast<float*>(q); };
    stem_bwd(reinterpret_cast<const void*>(x), reinterpret_cast<const void*>(c), reinterpret_cast<const void*>(dp),
             reinterpret_cast<const uint8_t*>(idx), F(w), F(mean), F(inv), W(part), blocks, W(stats), W(dw_bn),
             W(db_bn), W(dwp), n, reinterpret_cast<hipStream_t>(stream));
  });
  m.def("maxpool_bwd", [](uintptr_t dy, uintptr_t idx, uintptr_t dx, int64_t N, int64_t H, int64_t W, int64_t C,
                          int K, int S, int P, int dtype, uintptr_t stream) {
    maxpool_bwd(reinterpret_cast<const void*>(dy), reinterpret_cast<const uint8_t*>(idx), reinterpret_cast<void*>(dx),
                N, H, W, C, K, S, P, dtype, reinterpret_cast<hipStream_t>(stream));
  });

  // ---- Anderson solver (DEQ) ---------------------------------------------------
  m.def("anderson_gram_chunks", &anderson_gram_chunks);
  m.def("anderson_gram", [](uintptr_t X, uintptr_t F, int fdt, uintptr_t G, unsigned fresh, uintptr_t part,
                            int64_t bsz, int64_t d, int64_t rs, int64_t bs, int n, int last, int chunks,
                            uintptr_t stream, int hdt) {
    anderson_gram(reinterpret_cast<const void*>(X), reinterpret_cast<const void*>(F), fdt, reinterpret_cast<void*>(G),
                  fresh, reinterpret_cast<float*>(part), bsz, d, rs, bs, n, last, chunks, S(stream), hdt);
  }, py::arg("X"), py::arg("F"), py::arg("fdt"), py::arg("G"), py::arg("fresh"), py::arg("part"), py::arg("bsz"),
     py::arg("d"), py::arg("rs"), py::arg("bs"), py::arg("n"), py::arg("last"), py::arg("chunks"), py::arg("stream"),
     py::arg("hdt") = 7);
  m.def("adjoint_step_blocks", &adjoint_step_blocks);
  m.def("adjoint_step", [](uintptr_t vjp, uintptr_t grad, uintptr_t u, uintptr_t u_new, uintptr_t part, int blocks,
                           int64_t n, int dtype, uintptr_t stream) {
    adjoint_step(reinterpret_cast<const void*>(vjp), reinterpret_cast<const void*>(grad),
                 reinterpret_cast<const void*>(u), reinterpret_cast<void*>(u_new), reinterpret_cast<float*>(part),
                 blocks, n, dtype, S(stream));
  });
  m.def("anderson_solve", [](uintptr_t part, int chunks, int64_t bsz, int n, int last, float lam, uintptr_t alpha,
                             uintptr_t res, uintptr_t stream) {
    anderson_solve(reinterpret_cast<const float*>(part), chunks, bsz, n, last, lam, reinterpret_cast<float*>(alpha),
                   reinterpret_cast<float*>(res), S(stream));
  });
  m.def("anderson_mix", [](uintptr_t X, uintptr_t F, int fdt, uintptr_t alpha, uintptr_t z, int zdt, int64_t bsz,
                           int64_t d, int64_t rs, int64_t bs, int n, int slot, float beta, uintptr_t stream, int hdt) {
    anderson_mix(reinterpret_cast<void*>(X), reinterpret_cast<const void*>(F), fdt, reinterpret_cast<const float*>(alpha),
                 reinterpret_cast<void*>(z), zdt, bsz, d, rs, bs, n, slot, beta, S(stream), hdt);
  }, py::arg("X"), py::arg("F"), py::arg("fdt"), py::arg("alpha"), py::arg("z"), py::arg("zdt"), py::arg("bsz"),
     py::arg("d"), py::arg("rs"), py::arg("bs"), py::arg("n"), py::arg("slot"), py::arg("beta"), py::arg("stream"),
     py::arg("hdt") = 7);

  // ---- fused NHWC GroupNorm ------------------------------------------------------
  m.def("groupnorm_nhwc_fwd", [](uintptr_t x, uintptr_t a, uintptr_t h, uintptr_t y, uintptr_t w, uintptr_t b,
                                 uintptr_t mean, uintptr_t rstd, int64_t N, int64_t HW, int64_t C, int64_t G, bool relu,
                                 float eps, int dtype, uintptr_t stream, int64_t y_stride) {
    groupnorm_nhwc_fwd(reinterpret_cast<const void*>(x), reinterpret_cast<const void*>(a), reinterpret_cast<void*>(h),
                       reinterpret_cast<void*>(y), reinterpret_cast<const float*>(w), reinterpret_cast<const float*>(b),
                       reinterpret_cast<float*>(mean), reinterpret_cast<float*>(rstd), N, HW, C, G, relu, eps, dtype,
                       S(stream), y_stride);
  });
  m.def("groupnorm_nhwc_bwd", [](uintptr_t dy, uintptr_t h, uintptr_t mean, uintptr_t rstd, uintptr_t w, uintptr_t dh,
                                 uintptr_t part, int64_t N, int64_t HW, int64_t C, int64_t G, bool relu, int dtype,
                                 uintptr_t stream) {
    groupnorm_nhwc_bwd(reinterpret_cast<const void*>(dy), reinterpret_cast<const void*>(h),
                       reinterpret_cast<const float*>(mean), reinterpret_cast<const float*>(rstd),
                       reinterpret_cast<const float*>(w), reinterpret_cast<void*>(dh), reinterpret_cast<float*>(part), N,
                       HW, C, G, relu, dtype, S(stream));
  });

  // ---- the DEQ cell in one kernel ------------------------------------------------------
  m.def("deq_cell_supported", &deq_cell_supported);
  m.def("deq_cell_fwd", [](uintptr_t z, uintptr_t x, uintptr_t w1, uintptr_t w2, std::array<uintptr_t, 3> gw,
                           std::array<uintptr_t, 3> gb, uintptr_t out, uintptr_t out32, int64_t out32_stride,
                           std::array<uintptr_t, 3> h, std::array<uintptr_t, 3> mean, std::array<uintptr_t, 3> rstd,
                           int64_t N, int64_t H, int64_t W, int64_t C, int64_t G, float eps, uintptr_t stream,
                           int64_t out_stride) {
    const float* gwp[3];
    const float* gbp[3];
    void* hp[3];
    float* mp[3];
    float* rp[3];
    for (int i = 0; i < 3; ++i) {
      gwp[i] = reinterpret_cast<const float*>(gw[i]);
      gbp[i] = reinterpret_cast<const float*>(gb[i]);
      hp[i] = reinterpret_cast<void*>(h[i]);
      mp[i] = reinterpret_cast<float*>(mean[i]);
      rp[i] = reinterpret_cast<float*>(rstd[i]);
    }
    deq_cell_fwd(reinterpret_cast<const void*>(z), reinterpret_cast<const void*>(x), reinterpret_cast<const void*>(w1),
                 reinterpret_cast<const void*>(w2), gwp, gbp, reinterpret_cast<void*>(out),
                 reinterpret_cast<float*>(out32), out32_stride, hp, mp, rp, N, H, W, C, G, eps, S(stream), out_stride);
  });
  m.def("deq_cell_vjp", [](uintptr_t u, std::array<uintptr_t, 3> h, uintptr_t w2t, uintptr_t w1t,
                           std::array<uintptr_t, 3> gw, std::array<uintptr_t, 3> mean, std::array<uintptr_t, 3> rstd,
                           uintptr_t out, uintptr_t grad, uintptr_t ss_part, int64_t N, int64_t H, int64_t W,
                           int64_t C, int64_t G, uintptr_t stream) {
    const void* hp[3];
    const float* gwp[3];
    const float* mp[3];
    const float* rp[3];
    for (int i = 0; i < 3; ++i) {
      hp[i] = reinterpret_cast<const void*>(h[i]);
      gwp[i] = reinterpret_cast<const float*>(gw[i]);
      mp[i] = reinterpret_cast<const float*>(mean[i]);
      rp[i] = reinterpret_cast<const float*>(rstd[i]);
    }
    deq_cell_vjp(reinterpret_cast<const void*>(u), hp, reinterpret_cast<const void*>(w2t),
                 reinterpret_cast<const void*>(w1t), gwp, mp, rp, reinterpret_cast<void*>(out),
                 reinterpret_cast<const void*>(grad), reinterpret_cast<float*>(ss_part), N, H, W, C, G, S(stream));
  });
  m.def("deq_adjoint_check", [](uintptr_t part, int64_t n, uintptr_t thresh2, uintptr_t ss_out, uintptr_t flag,
                                uintptr_t stream) {
    deq_adjoint_check(reinterpret_cast<const float*>(part), n, reinterpret_cast<const float*>(thresh2),
                      reinterpret_cast<float*>(ss_out), reinterpret_cast<float*>(flag), S(stream));
  });

  // ---- GELU backward + bias gradient -------------------------------------------------
  m.def("gelu_bwd_bias_blocks", &gelu_bwd_bias_blocks);
  m.def("colsum_blocks", &colsum_blocks);
  m.def("emulate_comm", [](int blocks, double us, uintptr_t stream, int threads, int lds) {
    emulate_comm(blocks, us, S(stream), threads, lds);
  });
  m.def("wgrad256_supported", &wgrad256_supported);
  m.def("wgrad256_actual_splits", &wgrad256_actual_splits);
  m.def("wgrad256_set_variant", &wgrad256_set_variant);
  m.def("gemm_wgrad256", [](uintptr_t a, uintptr_t b, uintptr_t ws, int64_t lda, int64_t ldb, int64_t M, int64_t N,
                            int64_t K, int splits, uintptr_t stream) {
    gemm_wgrad256(reinterpret_cast<const void*>(a), reinterpret_cast<const void*>(b), reinterpret_cast<float*>(ws), lda,
                  ldb, M, N, K, splits, S(stream));
  });
  m.def("gemm_nt_supported", &gemm_nt_supported);
  m.def("gemm_nt_colpart_rows", &gemm_nt_colpart_rows);
  m.def("gemm_nt_set_split", &gemm_nt_set_split);
  m.def("gemm_nt_get_split", &gemm_nt_get_split);
  m.def("gemm_nt", [](uintptr_t a, uintptr_t b, uintptr_t c, uintptr_t c2, uintptr_t bias, int bias_f32, uintptr_t h,
                      uintptr_t colpart, int64_t lda, int64_t ldb, int64_t ldc,
                      int64_t M, int64_t N, int64_t K, int epi, uintptr_t stream) {
    gemm_nt(reinterpret_cast<const void*>(a), reinterpret_cast<const void*>(b), reinterpret_cast<void*>(c),
            reinterpret_cast<void*>(c2), reinterpret_cast<const void*>(bias), bias_f32, reinterpret_cast<const void*>(h),
            reinterpret_cast<float*>(colpart), nullptr, lda, ldb, ldc, M, N, K, epi, S(stream));
  });
  m.def("gemm_nt_stats", [](uintptr_t a, uintptr_t b, uintptr_t c, uintptr_t stats, int64_t lda, int64_t ldb,
                            int64_t ldc, int64_t M, int64_t N, int64_t K, uintptr_t stream) {
    gemm_nt(reinterpret_cast<const void*>(a), reinterpret_cast<const void*>(b), reinterpret_cast<void*>(c), nullptr,
            nullptr, 0, nullptr, nullptr, reinterpret_cast<float*>(stats), lda, ldb, ldc, M, N, K, 3, S(stream));
  });
  m.def("linear_bwd_supported", &linear_bwd_supported);
  m.def("linear_bwd_splits", &linear_bwd_splits);
  m.def("linear_bwd", [](uintptr_t dy, uintptr_t x, uintptr_t w, uintptr_t dx, uintptr_t ws, int64_t M, int64_t N,
                         int64_t K, int64_t ldy, int64_t ldx, int64_t ldw, int64_t lddx, int splits, int dg_first,
                         uintptr_t stream) {
    linear_bwd(reinterpret_cast<const void*>(dy), reinterpret_cast<const void*>(x), reinterpret_cast<const void*>(w),
               reinterpret_cast<void*>(dx), reinterpret_cast<float*>(ws), M, N, K, ldy, ldx, ldw, lddx, splits, dg_first,
               S(stream));
  });
  m.def("conv_c3_supported", &conv_c3_supported);
  m.def("conv_c3_wgrad_blocks", &conv_c3_wgrad_blocks);
  m.def("conv_c3_fwd", [](uintptr_t x, uintptr_t w, uintptr_t y, int64_t N, int H, int W, int stride, int Cout,
                          uintptr_t stream) {
    conv_c3_fwd(reinterpret_cast<const void*>(x), reinterpret_cast<const void*>(w), reinterpret_cast<void*>(y), N, H,
                W, stride, Cout, S(stream));
  });
  m.def("conv_c3_wgrad", [](uintptr_t x, uintptr_t dy, uintptr_t part, int64_t N, int H, int W, int stride, int Cout,
                            uintptr_t stream) {
    conv_c3_wgrad(reinterpret_cast<const void*>(x), reinterpret_cast<const void*>(dy), reinterpret_cast<float*>(part),
                  N, H, W, stride, Cout, S(stream));
  });
  m.def("conv3x3n_supported", &conv3x3n_supported);
  m.def("conv3x3n_slots128", &conv3x3n_slots128);
  m.def("conv3x3n", [](uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t stats, int64_t pixels, int H, int W, int C,
                       int Cout, int epi, uintptr_t stream) {
    conv3x3n(reinterpret_cast<const void*>(x), reinterpret_cast<const void*>(w), reinterpret_cast<void*>(y),
             reinterpret_cast<float*>(stats), pixels, H, W, C, Cout, epi, S(stream));
  });
  m.def("wgrad3x3n_supported", &wgrad3x3n_supported);
  m.def("wgrad3x3n_splits", &wgrad3x3n_splits);
  m.def("wgrad3x3n_groups", &wgrad3x3n_groups);
  m.def("wgrad3x3n", [](uintptr_t dy, uintptr_t x, uintptr_t ws, int64_t N, int H, int W, int C, int Cout, int splits,
                        int variant, uintptr_t stream) {
    wgrad3x3n(reinterpret_cast<const void*>(dy), reinterpret_cast<const void*>(x), reinterpret_cast<float*>(ws), N, H,
              W, C, Cout, splits, variant, S(stream));
  });
  m.def("gemm_nt_conv_supported", &gemm_nt_conv_supported);
  m.def("gemm_nt_conv", [](uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t stats, int64_t nimg, int H, int W, int C,
                           int64_t Cout, int epi, uintptr_t stream, uintptr_t residual) {
    gemm_nt_conv(reinterpret_cast<const void*>(x), reinterpret_cast<const void*>(w), reinterpret_cast<void*>(y),
                 reinterpret_cast<float*>(stats), nimg, H, W, C, Cout, epi, S(stream),
                 reinterpret_cast<const void*>(residual));
  });
  m.def("transpose_bf16", [](uintptr_t src, uintptr_t dst, int64_t rows, int64_t cols, int64_t lds, int64_t ldd,
                             uintptr_t stream) {
    transpose_bf16(reinterpret_cast<const void*>(src), reinterpret_cast<void*>(dst), rows, cols, lds, ldd, S(stream));
  });
  m.def("colsum", [](uintptr_t x, uintptr_t part, int blocks, int64_t rows, int64_t N, int dtype, uintptr_t stream) {
    colsum(reinterpret_cast<const void*>(x), reinterpret_cast<float*>(part), blocks, rows, N, dtype, S(stream));
  });
  m.def("gelu_bwd_bias", [](uintptr_t dy, uintptr_t h, uintptr_t dh, uintptr_t part, int blocks, int64_t rows,
                            int64_t N, int dtype, uintptr_t stream) {
    gelu_bwd_bias(reinterpret_cast<const void*>(dy), reinterpret_cast<const void*>(h), reinterpret_cast<void*>(dh),
                  reinterpret_cast<float*>(part), blocks, rows, N, dtype, S(stream));
  });

  m.def("gelu_set_form", &gelu_set_form);
  m.def("gelu_fwd", [](uintptr_t h, uintptr_t g, int64_t n, int dtype, uintptr_t stream) {
    gelu_fwd(reinterpret_cast<const void*>(h), reinterpret_cast<void*>(g), n, dtype, S(stream));
  });
  m.def("gelu_form", &gelu_form);

  // ---- fused LayerNorm ------------------------------------------------------
  m.def("layernorm_fwd", [](uintptr_t x, uintptr_t res, uintptr_t h, uintptr_t y, uintptr_t w, uintptr_t b,
                            uintptr_t mean, uintptr_t rstd, int64_t rows, int64_t D, float eps, int dtype,
                            int wdtype, uintptr_t stream) {
    layernorm_fwd(reinterpret_cast<const void*>(x), reinterpret_cast<const void*>(res), reinterpret_cast<void*>(h),
                  reinterpret_cast<void*>(y), reinterpret_cast<const void*>(w), reinterpret_cast<const void*>(b),
                  reinterpret_cast<float*>(mean), reinterpret_cast<float*>(rstd), rows, D, eps, dtype, wdtype,
                  S(stream));
  });
  m.def("layernorm_bwd", [](uintptr_t dy, uintptr_t x, uintptr_t dh, uintptr_t mean, uintptr_t rstd, uintptr_t w,
                            uintptr_t dx, uintptr_t part, int max_blocks, int64_t rows, int64_t D, int dtype,
                            int wdtype, uintptr_t stream, bool colsum) {
    return layernorm_bwd(reinterpret_cast<const void*>(dy), reinterpret_cast<const void*>(x),
                         reinterpret_cast<const void*>(dh), reinterpret_cast<const float*>(mean),
                         reinterpret_cast<const float*>(rstd), reinterpret_cast<const void*>(w),
                         reinterpret_cast<void*>(dx), reinterpret_cast<float*>(part), max_blocks, rows, D, dtype,
                         wdtype, colsum, S(stream));
  });

  // ---- MFMA GEMM (1x1 conv) -------------------------------------------------
  m.def("gemm_bf16",
        [](uintptr_t a, uintptr_t b, uintptr_t c, int64_t lda, int64_t ldb, int64_t ldc, int64_t M, int64_t N,
           int64_t K, bool a_kmajor, bool b_kmajor, int mode, int splits, uintptr_t a_scale, uintptr_t a_shift,
           uintptr_t b_scale, uintptr_t b_shift, uintptr_t stats, int tile_m, int tile_n, uintptr_t stream, int nbuf, uintptr_t res, int64_t ldr,
           uintptr_t bnb_x, uintptr_t bnb_w, uintptr_t bnb_b, uintptr_t bnb_mean, uintptr_t bnb_inv,
           uintptr_t bnb_mask, int bnb_rm, int conv_h, int conv_w, int conv_c, int engine, uintptr_t res_mask,
           int res_sub_h, int res_sub_w, int a_sub_h, int a_sub_w, int conv_s) {
          GemmProblem g{reinterpret_cast<const void*>(a), reinterpret_cast<const void*>(b),
                        reinterpret_cast<void*>(c), lda, ldb, ldc, M, N, K, a_kmajor, b_kmajor, mode, splits,
                        reinterpret_cast<const float*>(a_scale), reinterpret_cast<const float*>(a_shift),
                        reinterpret_cast<const float*>(b_scale), reinterpret_cast<const float*>(b_shift),
                        reinterpret_cast<float*>(stats), tile_m, tile_n, nbuf,
                        reinterpret_cast<const void*>(res), ldr, reinterpret_cast<const void*>(bnb_x),
                        reinterpret_cast<const float*>(bnb_w), reinterpret_cast<const float*>(bnb_b),
                        reinterpret_cast<const float*>(bnb_mean), reinterpret_cast<const float*>(bnb_inv),
                        reinterpret_cast<const uint8_t*>(bnb_mask), bnb_rm, conv_h, conv_w, conv_c, engine,
                        reinterpret_cast<const uint8_t*>(res_mask), res_sub_h, res_sub_w, a_sub_h, a_sub_w, conv_s};
          gemm_bf16(g, S(stream));
        },
        py::arg("a"), py::arg("b"), py::arg("c"), py::arg("lda"), py::arg("ldb"), py::arg("ldc"), py::arg("M"),
        py::arg("N"), py::arg("K"), py::arg("a_kmajor"), py::arg("b_kmajor"), py::arg("mode"), py::arg("splits"),
        py::arg("a_scale"), py::arg("a_shift"), py::arg("b_scale"), py::arg("b_shift"), py::arg("stats"),
        py::arg("tile_m"), py::arg("tile_n"), py::arg("stream"), py::arg("nbuf") = 0, py::arg("res") = 0,
        py::arg("ldr") = 0, py::arg("bnb_x") = 0, py::arg("bnb_w") = 0, py::arg("bnb_b") = 0,
        py::arg("bnb_mean") = 0, py::arg("bnb_inv") = 0, py::arg("bnb_mask") = 0, py::arg("bnb_rm") = 0,
        py::arg("conv_h") = 0, py::arg("conv_w") = 0, py::arg("conv_c") = 0, py::arg("engine") = 0,
        py::arg("res_mask") = 0, py::arg("res_sub_h") = 0, py::arg("res_sub_w") = 0, py::arg("a_sub_h") = 0,
        py::arg("a_sub_w") = 0, py::arg("conv_s") = 1);

  m.def("gemm_wgrad",
        [](uintptr_t a, uintptr_t b, uintptr_t ws, int64_t lda, int64_t ldb, int64_t M, int64_t N, int64_t K,
           int splits, int conv_h, int conv_w, int conv_c, uintptr_t stream, int variant, int b_sub) {
          gemm_wgrad(reinterpret_cast<const void*>(a), reinterpret_cast<const void*>(b), reinterpret_cast<float*>(ws),
                     lda, ldb, M, N, K, splits, conv_h, conv_w, conv_c, S(stream), variant, b_sub);
        },
        py::arg("a"), py::arg("b"), py::arg("ws"), py::arg("lda"), py::arg("ldb"), py::arg("M"), py::arg("N"),
        py::arg("K"), py::arg("splits"), py::arg("conv_h") = 0, py::arg("conv_w") = 0, py::arg("conv_c") = 0,
        py::arg("stream") = 0, py::arg("variant") = 0, py::arg("b_sub") = 0);

  m.def("transpose_filters",
        [](const std::vector<uintptr_t>& src, const std::vector<uintptr_t>& dst, const std::vector<int>& co,
           const std::vector<int>& ci, const std::vector<int>& taps, uintptr_t stream) {
          transpose_filters(src, dst, co, ci, taps, S(stream));
        },
        py::arg("src"), py::arg("dst"), py::arg("co"), py::arg("ci"), py::arg("taps"), py::arg("stream"));

  m.def("gemm_splitk_reduce_seg", [](uintptr_t ws, int splits, int64_t n, int64_t seg, uintptr_t o0, uintptr_t o1,
                                     uintptr_t o2, int out_dtype, uintptr_t stream) {
    gemm_splitk_reduce_seg(reinterpret_cast<const float*>(ws), splits, n, seg, reinterpret_cast<void*>(o0),
                           reinterpret_cast<void*>(o1), reinterpret_cast<void*>(o2), out_dtype, S(stream));
  });
  m.def("gemm_splitk_reduce",
        [](uintptr_t ws, int splits, int64_t n, uintptr_t out, int out_dtype, uintptr_t stream) {
          gemm_splitk_reduce(reinterpret_cast<const float*>(ws), splits, n, reinterpret_cast<void*>(out), out_dtype,
                             S(stream));
        },
        py::arg("ws"), py::arg("splits"), py::arg("n"), py::arg("out"), py::arg("out_dtype"), py::arg("stream"));

  // ---- RCCL ----------------------------------------------------------------
  m.def("rccl_unique_id", []() { return py::bytes(rccl_unique_id()); });
  m.def("rccl_version", &rccl_version);
  py::class_<RcclComm>(m, "RcclComm")
      .def(py::init<const std::string&, int, int, int>(), py::call_guard<py::gil_scoped_release>())
      .def("allreduce", &RcclComm::allreduce, py::call_guard<py::gil_scoped_release>())
      .def("allreduce_many", &RcclComm::allreduce_many, py::call_guard<py::gil_scoped_release>())
      .def("broadcast", &RcclComm::broadcast, py::call_guard<py::gil_scoped_release>())
      .def("reduce", &RcclComm::reduce, py::call_guard<py::gil_scoped_release>())
      .def("allgather", &RcclComm::allgather, py::call_guard<py::gil_scoped_release>())
      .def("reduce_scatter", &RcclComm::reduce_scatter, py::call_guard<py::gil_scoped_release>())
      .def("alltoall", &RcclComm::alltoall, py::call_guard<py::gil_scoped_release>())
      .def("comm_count", &RcclComm::comm_count, py::call_guard<py::gil_scoped_release>())
      .def("comm_user_rank", &RcclComm::comm_user_rank, py::call_guard<py::gil_scoped_release>())
      .def("comm_device", &RcclComm::comm_device, py::call_guard<py::gil_scoped_release>())
      .def("async_error", &RcclComm::async_error, py::call_guard<py::gil_scoped_release>())
      .def_static("error_string", &RcclComm::error_string)
      .def("abort", &RcclComm::abort, py::arg("abort_wait_ms") = 2000, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("aborted", &RcclComm::aborted)
      .def_property_readonly("is_open", &RcclComm::is_open)
      .def("destroy", &RcclComm::destroy, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("size", &RcclComm::size)
      .def_property_readonly("device", &RcclComm::device);
}
