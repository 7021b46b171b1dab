/*
 * rwkvtts_codec_layout.h -- packed f32 weight layout of the BiCodec decoder (SparkTTS
 * BiCodec.detokenize: FVQ codebook + out_proj, FSQ speaker tokens -> d-vector, Vocos/ConvNeXt
 * prenet conditioned by AdaLN on the d-vector, DAC-style WaveGenerator with Snake activations).
 * The ONNX graph (BiCodecDetokenize.onnx) is absent from the reference tree, so this layout is
 * the assumed architecture of SURVEY §8a-7; weights are synthetic. Conv weights are stored
 * [out][tap][in]; a ConvTranspose1d weight (PyTorch [in][out][K]) is stored [out][K][in].
 */
#ifndef RWKVTTS_CODEC_LAYOUT_H
#define RWKVTTS_CODEC_LAYOUT_H
#include <stdint.h>
#include "rwkvtts.h"

enum {
  CD_CODEBOOK = 0, CD_OUTP_W, CD_OUTP_B,                 /* semantic FVQ */
  CD_FSQ_W, CD_FSQ_B, CD_SPK_W, CD_SPK_B,                /* speaker d-vector */
  CD_PRE_W, CD_PRE_B, CD_EMB_W, CD_EMB_B,                /* prenet in */
  CD_N0_SW, CD_N0_SB, CD_N0_HW, CD_N0_HB,                /* AdaLN after embed: scale/shift */
  CD_FLN_W, CD_FLN_B, CD_LIN_W, CD_LIN_B,                /* prenet out */
  CD_CIN_W, CD_CIN_B,                                    /* WaveGenerator conv_in */
  CD_SOUT_A, CD_COUT_W, CD_COUT_B,                       /* final snake + conv_out */
  CD_GLOBAL_COUNT
};
/* per ConvNeXt block */
enum { CB_DW_W = 0, CB_DW_B, CB_SW, CB_SB, CB_HW, CB_HB, CB_PW1_W, CB_PW1_B, CB_PW2_W, CB_PW2_B,
       CB_GAMMA, CB_COUNT };
/* per decoder up-block (snake, convT, 3 residual units) */
enum { CU_SNAKE = 0, CU_T_W, CU_T_B,
       CU_R0_A1, CU_R0_W7, CU_R0_B7, CU_R0_A2, CU_R0_W1, CU_R0_B1,
       CU_R1_A1, CU_R1_W7, CU_R1_B7, CU_R1_A2, CU_R1_W1, CU_R1_B1,
       CU_R2_A1, CU_R2_W7, CU_R2_B7, CU_R2_A2, CU_R2_W1, CU_R2_B1, CU_COUNT };
#define RWKVTTS_CODEC_SPK_LATENT 128

/* number of f32 elements of tensor t in group g (0 global, 1 prenet block, 2 up block) */
static inline int64_t rwkvtts_codec_numel(const rwkvtts_codec_dims* d, int g, int idx, int t) {
  const int64_t L = d->latent_dim, P = d->prenet_dim, I = d->prenet_inter, S = d->spk_dim;
  const int64_t Q = RWKVTTS_CODEC_SPK_LATENT;
  if (g == 0) {
    switch (t) {
      case CD_CODEBOOK: return (int64_t)d->codebook_size * d->codebook_dim;
      case CD_OUTP_W: return L * d->codebook_dim;
      case CD_OUTP_B: return L;
      case CD_FSQ_W: return Q * d->fsq_dims;
      case CD_FSQ_B: return Q;
      case CD_SPK_W: return S * Q * d->n_global;
      case CD_SPK_B: return S;
      case CD_PRE_W: return P * L;
      case CD_PRE_B: return P;
      case CD_EMB_W: return P * 7 * P;
      case CD_EMB_B: return P;
      case CD_N0_SW: case CD_N0_HW: return P * S;
      case CD_N0_SB: case CD_N0_HB: return P;
      case CD_FLN_W: case CD_FLN_B: return P;
      case CD_LIN_W: return L * P;
      case CD_LIN_B: return L;
      case CD_CIN_W: return (int64_t)d->dec_channels * 7 * L;
      case CD_CIN_B: return d->dec_channels;
      case CD_SOUT_A: return d->dec_channels >> d->n_up;
      case CD_COUT_W: return 7 * (int64_t)(d->dec_channels >> d->n_up);
      case CD_COUT_B: return 1;
    }
    return 0;
  }
  if (g == 1) {
    switch (t) {
      case CB_DW_W: return P * 7;
      case CB_SW: case CB_HW: return P * S;
      case CB_PW1_W: return I * P;
      case CB_PW1_B: return I;
      case CB_PW2_W: return P * I;
      default: return P;
    }
  }
  {
    const int64_t Ci = d->dec_channels >> idx, Co = d->dec_channels >> (idx + 1);
    switch (t) {
      case CU_SNAKE: return Ci;
      case CU_T_W: return Co * d->up_kernels[idx] * Ci;
      case CU_R0_W7: case CU_R1_W7: case CU_R2_W7: return Co * 7 * Co;
      case CU_R0_W1: case CU_R1_W1: case CU_R2_W1: return Co * Co;
      default: return Co;
    }
  }
}

/* element offset of (g, idx, t); g == -1 returns the total element count */
static inline int64_t rwkvtts_codec_offset(const rwkvtts_codec_dims* d, int g, int idx, int t) {
  int64_t off = 64; /* header: 64 floats (dims copy) */
  for (int gg = 0; gg < 3; ++gg) {
    const int nidx = gg == 0 ? 1 : (gg == 1 ? d->prenet_layers : d->n_up);
    const int nt = gg == 0 ? CD_GLOBAL_COUNT : (gg == 1 ? CB_COUNT : CU_COUNT);
    for (int i = 0; i < nidx; ++i)
      for (int tt = 0; tt < nt; ++tt) {
        if (gg == g && i == idx && tt == t) return off;
        off += (rwkvtts_codec_numel(d, gg, i, tt) + 63) & ~(int64_t)63;
      }
  }
  return off;
}
#endif
