// Error plumbing + version for libstx (host side).
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stddef.h>
#include <stdio.h>

#include "../../include/stx.h"

namespace stx {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return (int)e;
  }
  return STX_OK;
}

}  // namespace stx

extern "C" int stx_version(void) { return 1; }
extern "C" const char* stx_last_error_string(void) { return stx::g_err; }
extern "C" int stx_abi_version(void) { return STX_ABI_VERSION; }

// sizeof and the offset of the last member of each ABI struct (include/stx.h order), for
// bindings to check their struct mirrors against: a member added on one side only moves
// one of these
extern "C" int stx_abi_layout(long long* out, int n) {
  const long long v[] = {
      (long long)sizeof(stx_conv_params),  (long long)offsetof(stx_conv_params, unpool_out),
      (long long)sizeof(stx_wprep_job),    (long long)offsetof(stx_wprep_job, pad_),
      (long long)sizeof(stx_loss_parts),   (long long)offsetof(stx_loss_parts, k),
      (long long)sizeof(stx_gram_fin_job), (long long)offsetof(stx_gram_fin_job, coef_amax),
      (long long)sizeof(stx_in_pgrad_job), (long long)offsetof(stx_in_pgrad_job, pad_),
      (long long)sizeof(stx_image_meta),   (long long)offsetof(stx_image_meta, tmp_offset)};
  const int m = (int)(sizeof(v) / sizeof(v[0]));
  for (int i = 0; out && i < n && i < m; ++i) out[i] = v[i];
  return m;
}
