// Host interface of the direct 3x3 convolution for small channel counts (conv_direct.hip),
// dispatched from yms_conv_fwd / yms_conv_dgrad / yms_conv_stats_rows in conv_igemm.hip.
#pragma once
#include "yms_common.hpp"

namespace yms {

struct DirectGeo {
  int TW, TH;            // output tile (TW divides the map width)
  int CP;                // 16-B chunks of reduction channels per pixel (4 or 8)
  int NCF;               // 32-column MFMA fragments of output channels (1 or 2)
  bool S2;               // stride-2 input gradient (tiles of class positions)
  int tiles_x, tiles_y;
  long ntiles;
  int grid;              // persistent blocks (= statistics rows of a training forward)
};

// True when the direct kernel runs this conv: 16-bit, 3x3, pad 1, reduction channels rounded to
// 8 of 32 or 64, at most 64 output channels (a multiple of 8), map width a multiple of 16.
// mode 0 = stride-1 forward (reduction = cin), 1 = input gradient (reduction = cout) of a stride-1
// conv, or of a stride-2 conv by output parity class (grid width ceil(w / 2) a multiple of 16).
// Off when YMS_DIRECT=0 at the first call or after yms_conv_direct_set(0) (A/B and tests).
// bnred: the input gradient with the producer's BN-reduce epilogue (yms_conv_dgrad_bnred): <= 32
// dx channels, one block per CU (its grid = the partial-row count).
bool conv_direct_geometry(const yms_conv_shape* s, int mode, DirectGeo* g, bool bnred = false);

// The producer's BN + act backward reduce fused into an input gradient's epilogue (yms_conv_dgrad_bnred):
// z view of the dx pixels, its BN scale / shift / [mean | invstd], act, partial rows ws[grid][2][cin].
struct DirectBnRed {
  const void* z;
  int z_ld, z_off;
  const float* scale;
  const float* shift;
  const float* mean_invstd;
  int act;
  float* ws;
};

yms_status conv_direct_launch(const yms_conv_shape* s, int mode, const DirectGeo& g, const void* src, int src_ld,
                              int src_off, const void* wpacked, void* dst, int dst_ld, int dst_off,
                              const float* scale, const float* shift, int act, const void* res, int res_ld,
                              int res_off, float* stats, int accumulate, hipStream_t st,
                              const DirectBnRed* bnr = nullptr);

}  // namespace yms
