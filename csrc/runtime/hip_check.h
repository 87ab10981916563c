#pragma once
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#define HIP_CHECK(x)                                                                         \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess)                                                                    \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e_) + " (" #x \
                               ") at " + __FILE__ + ":" + std::to_string(__LINE__));          \
  } while (0)
