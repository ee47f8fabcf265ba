// Host interface of the halo-tiled 3x3 weight gradient (wgrad_halo.hip), dispatched from
// yms_conv_wgrad / yms_conv_wgrad_ws_bytes in conv_igemm.hip.
#pragma once
#include "yms_common.hpp"

namespace yms {

struct WHPlan {
  int S, mb, nb, wk, kp, hb;          // kernel variant: stride, co / ci 32-blocks, k-step wave groups,
                                      // pixels and halo capacity
  int TW, R, HR, HC;                  // patch of R x TW output pixels, halo of HR x HC input pixels
  int ptx, pty, npatch, splits, pps;  // patches per row / column, total, splits over patches, per split
  int tiles_co, tiles_ci, slab_rows, slab_ld;
};

// False when the shape / dtype is not handled here (the im2col TT kernel runs instead) or
// YMS_WG_HALO=0.
bool wgrad_halo_plan(const yms_conv_shape* s, WHPlan* w);
// Partial slabs [splits * wk][slab_rows][9 * cin8] (the layout wgrad_reduce_kernel sums).
yms_status wgrad_halo_launch(const yms_conv_shape* s, const WHPlan& w, const void* x, int x_ld, int x_off,
                             const void* dz, int dz_ld, int dz_off, float* slab, hipStream_t st);

}  // namespace yms
