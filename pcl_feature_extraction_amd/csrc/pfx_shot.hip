// pfx_shot.hip -- SHOTEstimationOMP<PointXYZRGB,Normal,SHOT352> (placeholder until implemented)
#include "pfx_internal.h"
namespace pfx {
void shot_dev(pfx_ctx*, const float*, const float*, const float*, const float*, const float*, const float*,
              int64_t, const float*, const float*, const float*, int64_t, double, float*, float*) {
  throw Error(PFX_ERR_UNSUPPORTED, "shot: not implemented yet");
}
}  // namespace pfx
