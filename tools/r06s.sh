#!/bin/bash
# round-6 GPU call s: non-temporal loads on the last read of BN-streamed tensors (apply: gy, z; affine: z), interleaved A/B
set -e
O=gpurun_out/r06s; mkdir -p $O
bash tools/ab_train.sh $O/ab 3 "YMS_X=0|" "YMS_LIB=tools/bin/libyms_nt1.so|" "YMS_LIB=tools/bin/libyms_nt2.so|" "YMS_LIB=tools/bin/libyms_nt3.so|"
bash tools/ab_train.sh $O/ab_ms 2 "YMS_X=0|--version ms-s --steps 40" "YMS_LIB=tools/bin/libyms_nt1.so|--version ms-s --steps 40" "YMS_LIB=tools/bin/libyms_nt3.so|--version ms-s --steps 40"
echo done
