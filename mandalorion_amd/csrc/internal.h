// internal.h — helpers shared by the libmando translation units (not part of the public ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/mando.h"

namespace mando {
// records msg as the thread-local mando_last_error() text and returns code
int set_error(int code, const std::string &msg);
int ctx_device(const mando_ctx *ctx);
hipStream_t ctx_stream(const mando_ctx *ctx);
// a non-blocking stream on a hardware queue of its own (see capi.hip); the current device's
hipError_t create_stream(hipStream_t *out);
}  // namespace mando
