// Cross-rank sums of the sharded paths: the exact Vecchia rows' six partial sums
// and the latent path's probe-column statistics. Device buffers, ordered on the caller's stream.
//   RcclCollective          ncclAllReduce over xGMI (the production transport)
//   HostCallbackCollective  the buffer is copied to the host, summed by a caller-supplied
//                           function (e.g. a gloo all-reduce), and copied back — a test transport
//                           for several ranks sharing one GPU, where RCCL refuses to run.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <vector>

#include "common.h"

namespace gpb_amd {

class Collective {
 public:
  virtual ~Collective() = default;
  virtual void AllReduceSum(double* dev, int count, hipStream_t s) = 0;
};

class RcclCollective : public Collective {
 public:
  explicit RcclCollective(ncclComm_t c) : c_(c) {}
  void AllReduceSum(double* dev, int count, hipStream_t s) override {
    const ncclResult_t r = ncclAllReduce(dev, dev, count, ncclDouble, ncclSum, c_, s);
    if (r != ncclSuccess) Fatal("ncclAllReduce failed: %s", ncclGetErrorString(r));
  }

 private:
  ncclComm_t c_;
};

// fn(buf, count, user) must replace buf[0..count) by the element-wise sum over all ranks.
typedef void (*HostAllReduceFn)(double* buf, int count, void* user);

class HostCallbackCollective : public Collective {
 public:
  HostCallbackCollective(HostAllReduceFn fn, void* user) : fn_(fn), user_(user) {}
  void AllReduceSum(double* dev, int count, hipStream_t s) override {
    if (count <= 0) return;
    h_.resize(count);
    HIP_CHECK(hipMemcpyAsync(h_.data(), dev, sizeof(double) * count, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    fn_(h_.data(), count, user_);
    HIP_CHECK(hipMemcpyAsync(dev, h_.data(), sizeof(double) * count, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipStreamSynchronize(s));
  }

 private:
  HostAllReduceFn fn_;
  void* user_;
  std::vector<double> h_;
};

}  // namespace gpb_amd
