// Shared host-side utilities: error handling (reference c_api.cpp:54-58 semantics),
// logging (reference log.h:171-191 / LGBM_RegisterLogCallback), HIP checks.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <stdexcept>
#include <string>

namespace gpb_amd {

// Fatal error: thrown, caught at the C-ABI boundary, turned into -1 + LGBM_GetLastError.
[[noreturn]] void Fatal(const char* fmt, ...);
void Info(const char* fmt, ...);
void Warning(const char* fmt, ...);

#define HIP_CHECK(expr)                                                                 \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      ::gpb_amd::Fatal("HIP error '%s' at %s:%d (%s)", hipGetErrorString(_e), __FILE__, \
                       __LINE__, #expr);                                                \
  } while (0)

// Owning device buffer (hipMalloc/hipFree), no implicit copies.
template <typename T>
class DevBuf {
 public:
  DevBuf() = default;
  explicit DevBuf(size_t n) { alloc(n); }
  ~DevBuf() { release(); }
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p_(o.p_), n_(o.n_) { o.p_ = nullptr; o.n_ = 0; }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) { release(); p_ = o.p_; n_ = o.n_; o.p_ = nullptr; o.n_ = 0; }
    return *this;
  }
  void alloc(size_t n) {
    if (n == n_ && p_) return;
    release();
    if (n) HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&p_), n * sizeof(T)));
    n_ = n;
  }
  void release() {
    if (p_) (void)hipFree(p_);
    p_ = nullptr;
    n_ = 0;
  }
  T* get() const { return p_; }
  size_t size() const { return n_; }

 private:
  T* p_ = nullptr;
  size_t n_ = 0;
};

}  // namespace gpb_amd
