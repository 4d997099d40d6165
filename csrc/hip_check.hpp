// HIP error check for the GPU translation units (host builds never include
// it): a failing call goes through p2p::fatal, so abort hooks run (reference
// equivalent: CUDACHECK, p2p_matrix.cc:25-32, which exit()s one rank).
#pragma once

#include <hip/hip_runtime.h>

#include "common.hpp"

#define HIPCHECK(cmd)                                                                            \
  do {                                                                                           \
    hipError_t e_ = (cmd);                                                                       \
    if (e_ != hipSuccess) P2P_FATAL(::p2p::strfmt("HIP error in %s: %s", #cmd, hipGetErrorString(e_))); \
  } while (0)
