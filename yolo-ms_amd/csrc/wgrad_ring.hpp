// Host interface of the LDS-DMA ring weight gradient (wgrad_ring.hip), dispatched from
// yms_conv_wgrad / yms_conv_wgrad_ws_bytes in conv_igemm.hip.
#pragma once
#include "yms_common.hpp"

namespace yms {

struct WRPlan {
  int bm, bn, kp;                            // tile rows (co) / columns (tap*cin8+ci), pixels per k-tile
  int cin8, cpt, kc;                         // input channels rounded to 8, 16-B chunks per tap, valid chunks
  int tiles_m, tiles_n, nkt, kt_per_split, splits, slab_rows, slab_ld;
};

// False when the shape / dtype is not handled here (another weight-gradient kernel runs) or
// YMS_WG_RING=0.
bool wgrad_ring_plan(const yms_conv_shape* s, WRPlan* w);
// Partial slabs [splits][slab_rows][slab_ld] (the layout wgrad_reduce_kernel sums).
yms_status wgrad_ring_launch(const yms_conv_shape* s, const WRPlan& w, const void* x, int x_ld, int x_off,
                             const void* dz, int dz_ld, int dz_off, float* slab, hipStream_t st);

}  // namespace yms
