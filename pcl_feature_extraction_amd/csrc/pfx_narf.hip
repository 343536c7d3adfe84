// pfx_narf.hip -- RangeImagePlanar + RangeImageBorderExtractor + NarfKeypoint (placeholder)
#include "pfx_internal.h"
namespace pfx {
void range_image_dev(pfx_ctx*, const float*, const float*, const float*, int64_t, const pfx_camera&, float4*) {
  throw Error(PFX_ERR_UNSUPPORTED, "range image: not implemented yet");
}
int64_t narf_dev(pfx_ctx*, const float*, const float*, const float*, int64_t, const pfx_camera&,
                 const pfx_narf_params&, std::vector<int32_t>&) {
  throw Error(PFX_ERR_UNSUPPORTED, "narf: not implemented yet");
}
void narf_debug(pfx_ctx*, const std::string&, void*, int64_t) {
  throw Error(PFX_ERR_UNSUPPORTED, "narf: not implemented yet");
}
void narf_release(pfx_ctx*) {}
}  // namespace pfx
