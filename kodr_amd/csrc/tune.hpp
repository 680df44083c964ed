// Tuning knobs: environment switches that A/B measurements flip (tools/).
// The shipped build reads none of them -- each call site falls back to its
// measured default -- and only a tuning build (-DKODR_TUNE, implied by the
// -DKODR_TUNE_MODES / -DKODR_ELIM_TIMING probe builds) reads the environment.
// Runtime settings that stay in every build: KODR_POOL_BYTES (pool.hpp),
// KODR_HOST_THREADS (host_pool.hpp), KODR_ADD_TIMING (phase timing on stderr).
#pragma once
#include <stdlib.h>

#if defined(KODR_TUNE_MODES) || defined(KODR_ELIM_TIMING)
#ifndef KODR_TUNE
#define KODR_TUNE 1
#endif
#endif

namespace kodr_amd {
inline const char* tune_env(const char* name) {
#ifdef KODR_TUNE
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}
}  // namespace kodr_amd
