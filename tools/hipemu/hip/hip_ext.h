// hipemu (DEBUG-ONLY): hipExtLaunchKernelGGL -- the launch, with its start / stop events recorded
// around it on the host.
#pragma once
#include "hip_runtime.h"
#define hipExtLaunchKernelGGL(K, G, B, S, ST, E0, E1, F, ...)       \
  do {                                                              \
    if (E0) hipEventRecord((E0), (ST));                             \
    hipLaunchKernelGGL(K, G, B, S, ST, __VA_ARGS__);                \
    if (E1) hipEventRecord((E1), (ST));                             \
  } while (0)
