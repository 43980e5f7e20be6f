// pskv_frames.cpp — page-locked frame arena (see pskv_frames.h).
//
// Frames are hipHostMalloc'd (portable, mapped) in power-of-two size classes
// from 4 KiB up.  A frame moves between three states:
//   live    handed out by alloc; looked up by address (std::map over the
//           frame bases) when a call receives host pointers under
//           PSKV_HOST_FRAME
//   held    freed by the caller while work that reads it is still queued (one
//           event per queued use, recorded on the shard's stream)
//   cached  on its class's free list, reused by the next alloc of that class
// Free frames past the cache limit (PSKV_FRAME_CACHE_BYTES, default 1 GiB) go
// back to the system.  The arena is never destroyed: frames may be released
// from static destructors after the HIP runtime has begun to shut down.
#include "pskv_frames.h"

#include <cstdlib>
#include <map>
#include <mutex>
#include <vector>

#include "pskv.h"

namespace pskv {
namespace frames {
namespace {

constexpr int kMinLog = 12;  // 4 KiB: one page
constexpr int kClasses = 64;

struct Use {
  int device;
  hipEvent_t ev;
};

struct Frame {
  char* base;
  char* dev;  // device address of base
  size_t cap;
  int cls;
  std::vector<Use> uses;  // queued reads not yet known to have run
};

int size_class(size_t bytes) {
  int c = kMinLog;
  while (c < kClasses - 1 && (size_t(1) << c) < bytes) ++c;
  return c;
}

class Arena {
 public:
  static Arena& get() {
    static Arena* a = new Arena();  // never destroyed, see the file comment
    return *a;
  }

  int alloc(size_t bytes, void** out, std::string* err) {
    if (!out) return set(err, PSKV_EINVAL, "pskv_host_alloc: null out");
    *out = nullptr;
    if (bytes > (size_t(1) << 46)) return set(err, PSKV_EINVAL, "pskv_host_alloc: size too large");
    const int cls = size_class(bytes);
    Frame* f = nullptr;
    std::vector<Frame*> drop;
    {
      std::lock_guard<std::mutex> g(mu_);
      sweep_held(&drop);
      if (!free_[cls].empty()) {
        f = free_[cls].back();
        free_[cls].pop_back();
        cached_ -= f->cap;
      }
    }
    release_to_system(drop);
    if (!f) {
      const size_t cap = size_t(1) << cls;
      void* p = nullptr;
      hipError_t e = hipHostMalloc(&p, cap, hipHostMallocPortable | hipHostMallocMapped);
      if (e != hipSuccess) {
        (void)hipGetLastError();
        std::string ignore;
        (void)trim(&ignore);  // cached frames of other classes may be in the way
        e = hipHostMalloc(&p, cap, hipHostMallocPortable | hipHostMallocMapped);
        if (e != hipSuccess) {
          (void)hipGetLastError();
          return set(err, PSKV_ENOMEM, "pskv_host_alloc: page-locked allocation failed");
        }
      }
      void* dev = nullptr;
      if (hipHostGetDevicePointer(&dev, p, 0) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipHostFree(p);
        return set(err, PSKV_EHIP, "pskv_host_alloc: hipHostGetDevicePointer failed");
      }
      // The frame is portable (every device may map it), but a kernel reads it
      // in place only through ONE address for all devices: ROCm's unified
      // address space maps page-locked memory at its host address on every
      // device.  Should a device view ever differ from the host address, the
      // frame keeps no view and calls on it take the DMA path (device_view
      // returns null), which is correct for any device.
      f = new Frame{static_cast<char*>(p), dev == p ? static_cast<char*>(dev) : nullptr, cap, cls, {}};
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      live_[reinterpret_cast<uintptr_t>(f->base)] = f;
      live_bytes_ += f->cap;
    }
    *out = f->base;
    return PSKV_OK;
  }

  int release(void* p, std::string* err) {
    if (!p) return PSKV_OK;  // like free(NULL)
    std::vector<Frame*> drop;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = live_.find(reinterpret_cast<uintptr_t>(p));
      if (it == live_.end())
        return set(err, PSKV_EINVAL, "pskv_host_free: not a live frame (freed twice, or not from pskv_host_alloc)");
      Frame* f = it->second;
      live_.erase(it);
      live_bytes_ -= f->cap;
      prune(f);
      if (f->uses.empty()) {
        cache(f, &drop);
      } else {
        held_.push_back(f);
        held_bytes_ += f->cap;
      }
    }
    release_to_system(drop);
    return PSKV_OK;
  }

  void* device_view(const void* p, size_t bytes) {
    std::lock_guard<std::mutex> g(mu_);
    Frame* f = find(p);
    if (!f || !f->dev) return nullptr;
    const size_t off = static_cast<size_t>(static_cast<const char*>(p) - f->base);
    if (bytes > f->cap - off) return nullptr;
    return f->dev + off;
  }

  int note_use(const void* p, int device, hipStream_t st, std::string* err) {
    std::lock_guard<std::mutex> g(mu_);
    Frame* f = find(p);
    if (!f) return PSKV_OK;
    if (f->uses.size() >= 4) prune(f);  // a frame passed to many calls keeps few events
    hipEvent_t e = nullptr;
    auto& sp = spare_[device];
    if (!sp.empty()) {
      e = sp.back();
      sp.pop_back();
    } else if (hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence) !=
               hipSuccess) {
      (void)hipGetLastError();
      return set(err, PSKV_EHIP, "frame use: hipEventCreate failed");
    }
    if (hipEventRecord(e, st) != hipSuccess) {
      (void)hipGetLastError();
      sp.push_back(e);
      return set(err, PSKV_EHIP, "frame use: hipEventRecord failed");
    }
    f->uses.push_back(Use{device, e});
    return PSKV_OK;
  }

  void stats(uint64_t* live, uint64_t* cached, uint64_t* held) {
    std::vector<Frame*> drop;
    {
      std::lock_guard<std::mutex> g(mu_);
      sweep_held(&drop);
      if (live) *live = live_bytes_;
      if (cached) *cached = cached_;
      if (held) *held = held_bytes_;
    }
    release_to_system(drop);
  }

  int trim(std::string* err) {
    std::vector<Frame*> drop, wait;
    {
      std::lock_guard<std::mutex> g(mu_);
      wait.swap(held_);
      held_bytes_ = 0;
      for (auto& fl : free_) {
        for (Frame* f : fl) drop.push_back(f);
        fl.clear();
      }
      cached_ = 0;
    }
    int rc = PSKV_OK;
    for (Frame* f : wait) {
      for (const Use& u : f->uses) {
        if (hipEventSynchronize(u.ev) != hipSuccess) {
          (void)hipGetLastError();
          rc = set(err, PSKV_EHIP, "pskv_host_pool_trim: hipEventSynchronize failed");
        }
      }
      std::lock_guard<std::mutex> g(mu_);
      for (const Use& u : f->uses) spare_[u.device].push_back(u.ev);
      f->uses.clear();
      drop.push_back(f);
    }
    release_to_system(drop);
    return rc;
  }

 private:
  Arena() {
    if (const char* e = std::getenv("PSKV_FRAME_CACHE_BYTES")) max_cached_ = (size_t)std::atoll(e);
  }

  static int set(std::string* err, int code, const char* msg) {
    if (err) *err = msg;
    return code;
  }

  // the live frame whose bytes contain p (mu_ held)
  Frame* find(const void* p) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    auto it = live_.upper_bound(a);
    if (it == live_.begin()) return nullptr;
    --it;
    Frame* f = it->second;
    return a < it->first + f->cap ? f : nullptr;
  }

  // drop the uses whose events have completed (mu_ held)
  void prune(Frame* f) {
    size_t k = 0;
    for (const Use& u : f->uses) {
      const hipError_t q = hipEventQuery(u.ev);
      if (q == hipErrorNotReady) {
        f->uses[k++] = u;
      } else {
        if (q != hipSuccess) (void)hipGetLastError();  // a failed use reads nothing more
        spare_[u.device].push_back(u.ev);
      }
    }
    f->uses.resize(k);
  }

  // held frames whose reads have all run go to the cache (mu_ held)
  void sweep_held(std::vector<Frame*>* drop) {
    size_t k = 0;
    for (Frame* f : held_) {
      prune(f);
      if (f->uses.empty()) {
        held_bytes_ -= f->cap;
        cache(f, drop);
      } else {
        held_[k++] = f;
      }
    }
    held_.resize(k);
  }

  void cache(Frame* f, std::vector<Frame*>* drop) {
    if (cached_ + f->cap > max_cached_) {
      drop->push_back(f);
      return;
    }
    free_[f->cls].push_back(f);
    cached_ += f->cap;
  }

  static void release_to_system(std::vector<Frame*>& drop) {
    for (Frame* f : drop) {
      (void)hipHostFree(f->base);
      delete f;
    }
    drop.clear();
  }

  std::mutex mu_;
  std::map<uintptr_t, Frame*> live_;
  std::vector<Frame*> free_[kClasses];
  std::vector<Frame*> held_;
  std::map<int, std::vector<hipEvent_t>> spare_;  // recycled events by device
  size_t live_bytes_ = 0, cached_ = 0, held_bytes_ = 0;
  size_t max_cached_ = size_t(1) << 30;
};

}  // namespace

int alloc(size_t bytes, void** out, std::string* err) { return Arena::get().alloc(bytes, out, err); }
int release(void* p, std::string* err) { return Arena::get().release(p, err); }
void* device_view(const void* p, size_t bytes) { return Arena::get().device_view(p, bytes); }
int note_use(const void* p, int device, hipStream_t stream, std::string* err) {
  return Arena::get().note_use(p, device, stream, err);
}
void stats(uint64_t* live, uint64_t* cached, uint64_t* held) { Arena::get().stats(live, cached, held); }
int trim(std::string* err) { return Arena::get().trim(err); }

}  // namespace frames
}  // namespace pskv
