// Host interface of the halo-tiled 3x3 stride-1 convolution (conv_halo.hip), dispatched from the
// C-ABI entry points in conv_igemm.hip.
#pragma once
#include "yms_common.hpp"

namespace yms {

struct HaloGeo {
  int TW, TH, ntx, nty, tiles_m, tiles_n, bn, hp, nkc;
};

// mode 0 = forward, 1 = stride-1 input gradient.  False when the shape / dtype is not handled
// (the im2col NT kernel runs instead) or YMS_HALO=0.
bool conv_halo_geometry(const yms_conv_shape* s, int mode, HaloGeo* g);
yms_status conv_halo_launch(const yms_conv_shape* s, int mode, const HaloGeo& g, const void* src, int src_ld,
                            int src_off, const void* wpacked, void* dst, int dst_ld, int dst_off, const float* scale,
                            const float* shift, int act, const void* res, int res_ld, int res_off, float* stats,
                            int accumulate, hipStream_t st);

}  // namespace yms
