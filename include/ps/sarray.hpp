// ps/sarray.hpp — clean-room restatement of the reference's shared array
// (base/third_party/sarray.h) with only the behaviour the storage boundary
// relies on:
//   * shared ownership with a custom deleter          (sarray.h:95-101,168-171)
//   * zero-copy reinterpret SArray<W>(SArray<V>),
//     size = bytes / sizeof(W), truncated              (sarray.h:67-82)
//   * SArray<V>(n) is zero-filled                      (sarray.h:56,179-195)
//   * segment(b, e) is a zero-copy view                (sarray.h:269-275)
// Used by the standalone C++ build of the boundary (tests/cpp); inside the
// reference tree the reference's own SArray is used instead.
#pragma once

#include <cstddef>
#include <cstring>
#include <initializer_list>
#include <memory>
#include <vector>

namespace csci5570 {
namespace third_party {

template <typename V>
class SArray {
 public:
  SArray() = default;
  explicit SArray(size_t n) : size_(n) {
    if (n) {
      ptr_ = std::shared_ptr<V>(new V[n], [](V* p) { delete[] p; });
      std::memset(static_cast<void*>(ptr_.get()), 0, n * sizeof(V));
    }
  }
  SArray(V* data, size_t n, bool deletable = false) { reset_to(data, n, deletable); }
  template <typename D>
  void reset(V* data, size_t n, D deleter) {
    ptr_ = std::shared_ptr<V>(data, deleter);
    size_ = n;
  }
  template <typename W>
  explicit SArray(const SArray<W>& other) {
    *this = other;
  }
  template <typename W>
  SArray& operator=(const SArray<W>& other) {
    size_ = other.size() * sizeof(W) / sizeof(V);
    ptr_ = std::shared_ptr<V>(other.ptr(), reinterpret_cast<V*>(other.data()));
    return *this;
  }
  SArray(std::initializer_list<V> l) : SArray(l.size()) {
    size_t i = 0;
    for (const V& x : l) data()[i++] = x;
  }
  explicit SArray(const std::vector<V>& v) : SArray(v.size()) {
    if (!v.empty()) std::memcpy(static_cast<void*>(data()), v.data(), v.size() * sizeof(V));
  }

  size_t size() const { return size_; }
  bool empty() const { return size_ == 0; }
  V* data() const { return ptr_.get(); }
  const std::shared_ptr<V>& ptr() const { return ptr_; }
  V* begin() const { return data(); }
  V* end() const { return data() + size_; }
  V& operator[](size_t i) { return data()[i]; }
  const V& operator[](size_t i) const { return data()[i]; }

  SArray segment(size_t b, size_t e) const {
    SArray r;
    r.ptr_ = std::shared_ptr<V>(ptr_, data() + b);
    r.size_ = e - b;
    return r;
  }

 private:
  void reset_to(V* data, size_t n, bool deletable) {
    if (deletable)
      reset(data, n, [](V* p) { delete[] p; });
    else
      reset(data, n, [](V*) {});
  }
  size_t size_ = 0;
  std::shared_ptr<V> ptr_;
};

}  // namespace third_party
}  // namespace csci5570
