// fedcodec.hip — unity translation unit for libfedcodec.so (gfx950 only).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -shared fedcodec.hip
#include "fc_topk.hip"
#include "fc_pred.hip"
#include "fc_decode.hip"
#include "fc_qsgd.hip"
#include "fc_f64.hip"
#include "fc_capi.hip"
#include "fc_mt.hip"
