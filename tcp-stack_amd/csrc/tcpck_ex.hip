// tcpck_ex.hip -- the tuning entry points of libtcpck.so (include/tcpck_tuning.h):
// the product router with an explicit kernel / param and no measurement hooks.
// libtcpck_probe.so builds tcpck_ex_probe.hip in this file's place.
#include <hip/hip_runtime.h>

#include "tcpck.h"
#include "tcpck_tuning.h"
#include "tcpck_api_internal.h"

using tcpck::api::Hooks;

extern "C" {

int tcpck_batch_fixed_ex(tcpck_ctx *ctx, int op, int mode, void *d_arena, uint64_t stride, uint32_t len,
                         uint64_t count, void *d_out, int kernel, int param, tcpck_stream stream) {
  return tcpck::api::batch_fixed_ex(ctx, op, mode, d_arena, stride, len, count, d_out, kernel, param,
                                    static_cast<hipStream_t>(stream), Hooks{});
}

int tcpck_batch_var_ex(tcpck_ctx *ctx, int op, int mode, void *d_arena, const uint64_t *d_offsets,
                       const uint32_t *d_lengths, uint64_t count, void *d_out, const tcpck_layout *layout,
                       int kernel, int param, tcpck_stream stream) {
  return tcpck::api::batch_var_ex(ctx, op, mode, d_arena, d_offsets, d_lengths, count, d_out, layout, kernel, param,
                                  static_cast<hipStream_t>(stream), Hooks{});
}

int tcpck_batch_receive_ex(tcpck_ctx *ctx, int mode, void *d_arena, uint64_t stride, uint32_t len,
                           const uint64_t *d_offsets, const uint32_t *d_lengths, uint64_t count, uint8_t *d_ok,
                           void *d_hdr, const tcpck_layout *layout, int kernel, int param, tcpck_stream stream) {
  return tcpck::api::batch_receive_ex(ctx, mode, d_arena, stride, len, d_offsets, d_lengths, count, d_ok, d_hdr,
                                      layout, kernel, param, static_cast<hipStream_t>(stream), Hooks{});
}

}  // extern "C"
