// ps/svector.h — SVector<T>: a reference-counted array view, the container of
// every key / value / length array on the KV path (reference
// src/utility/SVector.h:119-620).
//
// Semantics kept from the reference: copies share the buffer (no data copy);
// construction from a std::vector copies; Slice() aliases a sub-range;
// reinterpreting SVector<U> -> SVector<T> shares the bytes; resize() grows in
// place when capacity allows, else detaches into a fresh buffer.
//
// MI355X addition: an SVector may live in HBM (device() >= 0).  Device arrays
// come from a per-GPU caching pool (internal/device.h) and are released back to
// it when the last SVector referencing them goes away.  Element access through
// operator[] / begin() is host-only; device arrays are consumed by the psg
// kernels (include/psg.h).
#pragma once
#include <algorithm>
#include <cstring>
#include <initializer_list>
#include <memory>
#include <sstream>
#include <string>
#include <type_traits>
#include <vector>

#include "ps/log.h"
#include "ps/range.h"

namespace ps {

namespace device {
// Pooled HBM allocation on `device` (implemented in src/device.cc).
std::shared_ptr<void> Alloc(size_t bytes, int device);
// Pooled pinned host block for a large host array, or nullptr (use the heap).
std::shared_ptr<void> HostAlloc(size_t bytes);
// Heap block on transparent huge pages for an array of >= 4 MiB (first touch
// faults 2 MiB at a time instead of 4 KiB), or nullptr.
std::shared_ptr<void> HugeAlloc(size_t bytes);
}  // namespace device

/* memcpy that splits copies of >= 16 MiB over several host threads (the
 * vector -> SVector copy of KVWorker::Push, the pull merge into the caller's
 * vector); implemented in src/device.cc. */
void HostCopy(void* dst, const void* src, size_t bytes);
/* memset split the same way (SVector::resize's zero fill of a large array) */
void HostFill(void* dst, int byte, size_t bytes);
/* first touch of a large host range the caller is about to overwrite (a
 * std::vector the Pull merge resizes): huge pages where the range allows, then
 * every page written in parallel, so the faults are not taken one 4 KiB page
 * at a time by one thread; a no-op below 4 MiB */
void PrefaultHost(void* p, size_t bytes);

template <typename T>
class SVector {
  static_assert(std::is_trivially_copyable<T>::value, "SVector holds trivially copyable types");
  template <typename U>
  friend class SVector;

 public:
  SVector() = default;
  ~SVector() = default;

  explicit SVector(size_t count) { resize(count); }
  SVector(size_t count, const T& value) { resize(count, value); }
  SVector(std::initializer_list<T> list) { CopyFrom(list.begin(), list.size()); }
  /* copies the vector (KVWorker::Push relies on this, KVApp.h:119-121) */
  explicit SVector(const std::vector<T>& vec) { CopyFrom(vec.data(), vec.size()); }
  /* shares the vector's storage */
  explicit SVector(const std::shared_ptr<std::vector<T>>& sp)
      : ptr_(sp, sp->data()), size_(sp->size()), capacity_(sp->capacity()) {}
  /* wraps a raw host array; owned (delete[]) only when deletable */
  SVector(T* data, size_t size, bool deletable = false) {
    if (deletable)
      ptr_ = std::shared_ptr<T>(data, [](T* p) { delete[] p; });
    else
      ptr_ = std::shared_ptr<T>(data, [](T*) {});
    size_ = capacity_ = size;
  }
  /* wraps a raw array with a custom deleter */
  template <typename Deleter>
  SVector(T* data, size_t size, Deleter d, int device = -1) : device_(device) {
    ptr_ = std::shared_ptr<T>(data, d);
    size_ = capacity_ = size;
  }

  SVector(const SVector& o) = default;
  SVector(SVector&& o) noexcept = default;
  SVector& operator=(const SVector& o) = default;
  SVector& operator=(SVector&& o) noexcept = default;

  /* reinterpret a SVector<U>: shares the bytes (SVector.h:155-207) */
  template <typename U, typename = std::enable_if_t<!std::is_same<U, T>::value>>
  SVector(const SVector<U>& o) {
    *this = o;
  }
  template <typename U, typename = std::enable_if_t<!std::is_same<U, T>::value>>
  SVector& operator=(const SVector<U>& o) {
    size_ = o.size_ * sizeof(U) / sizeof(T);
    capacity_ = o.capacity_ * sizeof(U) / sizeof(T);
    CHECK_EQ(size_ * sizeof(T), o.size_ * sizeof(U)) << "size should be divided";
    ptr_ = std::shared_ptr<T>(o.ptr_, reinterpret_cast<T*>(o.ptr_.get()));
    device_ = o.device_;
    return *this;
  }

  /* `count` host elements left uninitialised (a buffer a copy will fill) */
  static SVector Uninitialized(size_t count) {
    SVector v;
    v.reserve(count);
    v.size_ = count;
    return v;
  }

  /* ---- HBM arrays ---- */
  /* `count` uninitialised elements in the pool of GPU `device` */
  static SVector OnDevice(size_t count, int device) {
    SVector v;
    v.device_ = device;
    if (count) {
      auto p = device::Alloc(count * sizeof(T), device);
      v.ptr_ = std::shared_ptr<T>(p, static_cast<T*>(p.get()));
    }
    v.size_ = v.capacity_ = count;
    return v;
  }
  /* non-owning view of a device array */
  static SVector WrapDevice(T* dptr, size_t count, int device) {
    SVector v;
    v.device_ = device;
    v.ptr_ = std::shared_ptr<T>(dptr, [](T*) {});
    v.size_ = v.capacity_ = count;
    return v;
  }
  int device() const { return device_; }
  bool on_device() const { return device_ >= 0; }

  /* ---- access ---- */
  size_t size() const { return size_; }
  size_t capacity() const { return capacity_; }
  bool empty() const { return size_ == 0; }
  T* data() const { return ptr_.get(); }
  T* begin() { return data(); }
  const T* begin() const { return data(); }
  T* end() { return data() + size_; }
  const T* end() const { return data() + size_; }
  T& operator[](size_t i) const { return data()[i]; }
  T& front() const { return data()[0]; }
  T& back() const { return data()[size_ - 1]; }
  const std::shared_ptr<T>& ptr() const { return ptr_; }

  /* ---- modification (host arrays) ---- */
  void CopyFrom(const T* src, size_t n) {
    CHECK(!on_device()) << "CopyFrom into a device SVector";
    clear();
    reserve(n);
    size_ = n;
    if (n) HostCopy(data(), src, n * sizeof(T));
  }
  template <typename It>
  void CopyFrom(It first, It last) {
    std::vector<T> tmp(first, last);
    CopyFrom(tmp.data(), tmp.size());
  }

  void reserve(size_t n) {
    if (n <= capacity_) return;
    CHECK(!on_device()) << "reserve on a device SVector";
    std::shared_ptr<T> np;
    if (auto pinned = device::HostAlloc(n * sizeof(T)))  // large frames: pinned, PCIe-rate copies
      np = std::shared_ptr<T>(pinned, static_cast<T*>(pinned.get()));
    else if (auto huge = device::HugeAlloc(n * sizeof(T)))
      np = std::shared_ptr<T>(huge, static_cast<T*>(huge.get()));
    else  // left uninitialised: resize() fills what it adds, copies overwrite
      np = std::shared_ptr<T>(new T[n], [](T* p) { delete[] p; });
    if (size_) std::memcpy(np.get(), data(), size_ * sizeof(T));
    ptr_ = np;
    capacity_ = n;
  }
  void resize(size_t n, const T& val = T()) {
    size_t old = size_;
    if (n > capacity_) reserve(std::max(n, old * 2));
    if (n > old) {
      // a large zero fill (test_kv_app_benchmark's EmptyHandler answers a
      // Pull with res.vals.resize(n)) is split over the copy threads
      const T zero{};
      if (!on_device() && std::memcmp(&val, &zero, sizeof(T)) == 0)
        HostFill(data() + old, 0, (n - old) * sizeof(T));
      else
        std::fill(data() + old, data() + n, val);
    }
    size_ = n;
  }
  void clear() {
    if (ptr_ && ptr_.use_count() > 1) {  // detach from shared storage
      ptr_.reset();
      capacity_ = 0;
    }
    size_ = 0;
  }
  void push_back(const T& v) {
    if (size_ == capacity_) reserve(std::max<size_t>(8, capacity_ * 2));
    data()[size_++] = v;
  }
  void append(const SVector<T>& o) {
    size_t n = size_;
    resize(n + o.size());
    if (o.size()) std::memcpy(data() + n, o.data(), o.size() * sizeof(T));
  }

  /* [begin, end) view sharing the storage (SVector.h:302-312) */
  SVector Slice(size_t begin, size_t end) const {
    CHECK_LE(begin, end);
    CHECK_LE(end, size_);
    SVector r;
    r.ptr_ = std::shared_ptr<T>(ptr_, data() + begin);
    r.size_ = r.capacity_ = end - begin;
    r.device_ = device_;
    return r;
  }

  std::string DebugString() const {
    std::ostringstream os;
    os << "[" << size_ << (on_device() ? " @gpu" + std::to_string(device_) : "") << "]";
    if (!on_device()) {
      os << ":";
      for (size_t i = 0; i < std::min<size_t>(size_, 5); ++i) os << " " << +data()[i];
      if (size_ > 5) os << " ...";
    }
    return os.str();
  }

 private:
  std::shared_ptr<T> ptr_;
  size_t size_ = 0;
  size_t capacity_ = 0;
  int device_ = -1;
};

/* Index range of [lo, hi) inside the sorted array arr (SVector.h:670-676). */
template <typename T>
Range FindRange(const SVector<T>& arr, T lo, T hi) {
  if (arr.empty()) return Range(0, 0);
  auto lb = std::lower_bound(arr.begin(), arr.end(), lo);
  auto ub = std::lower_bound(arr.begin(), arr.end(), hi);
  return Range(lb - arr.begin(), ub - arr.begin());
}

}  // namespace ps
