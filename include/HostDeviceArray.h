// HostDeviceArray.h -- replaces QEC_LDPC/HostDeviceArray.h:6-39 (cusp/thrust
// typedefs plus a commented-out host+device pair) with a thin hipMalloc /
// hipHostMalloc / hipMemcpyAsync RAII wrapper.  Needs a HIP compiler
// (hipcc) because it calls the HIP runtime directly.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <stdexcept>
#include <string>
#include <vector>

// The reference's host container names (HostDeviceArray.h:6-13) as std::vector,
// so DecoderCPU-style call sites keep compiling.
typedef std::vector<int> IntArray1d_h;
typedef std::vector<float> FloatArray1d_h;

namespace qec {

inline void hip_throw(hipError_t e, const char* what)
{
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// Device buffer that only grows (reserve), so repeated batch calls reuse HBM.
template <class T>
class DeviceArray {
public:
    DeviceArray() = default;
    explicit DeviceArray(size_t n) { reserve(n); }
    DeviceArray(const DeviceArray&) = delete;
    DeviceArray& operator=(const DeviceArray&) = delete;
    DeviceArray(DeviceArray&& o) noexcept : p_(o.p_), cap_(o.cap_) { o.p_ = nullptr; o.cap_ = 0; }
    ~DeviceArray() { if (p_) (void)hipFree(p_); }
    void reserve(size_t n)
    {
        if (n <= cap_) return;
        if (p_) { (void)hipFree(p_); p_ = nullptr; cap_ = 0; }
        hip_throw(hipMalloc(reinterpret_cast<void**>(&p_), n * sizeof(T) + 16), "hipMalloc");
        cap_ = n;
    }
    T* data() { return p_; }
    const T* data() const { return p_; }
    size_t capacity() const { return cap_; }

private:
    T* p_ = nullptr;
    size_t cap_ = 0;
};

// Page-locked host buffer (so hipMemcpyAsync is truly asynchronous).
template <class T>
class PinnedArray {
public:
    PinnedArray() = default;
    explicit PinnedArray(size_t n) { reserve(n); }
    PinnedArray(const PinnedArray&) = delete;
    PinnedArray& operator=(const PinnedArray&) = delete;
    ~PinnedArray() { if (p_) (void)hipHostFree(p_); }
    void reserve(size_t n)
    {
        if (n <= cap_) return;
        if (p_) { (void)hipHostFree(p_); p_ = nullptr; cap_ = 0; }
        hip_throw(hipHostMalloc(reinterpret_cast<void**>(&p_), n * sizeof(T) + 16, hipHostMallocDefault), "hipHostMalloc");
        cap_ = n;
    }
    T* data() { return p_; }
    T& operator[](size_t i) { return p_[i]; }
    size_t capacity() const { return cap_; }

private:
    T* p_ = nullptr;
    size_t cap_ = 0;
};

// Host + device pair of one logical array (the commented HostDeviceArray1d,
// QEC_LDPC/HostDeviceArray.h:15-24), with explicit stream-ordered copies.
template <class T>
class HostDeviceArray {
public:
    explicit HostDeviceArray(size_t n = 0) : n_(n) { resize(n); }
    void resize(size_t n) { n_ = n; host_.reserve(n); dev_.reserve(n); }
    size_t size() const { return n_; }
    T* host() { return host_.data(); }
    T* device() { return dev_.data(); }
    void upload(hipStream_t s = nullptr)
    {
        hip_throw(hipMemcpyAsync(dev_.data(), host_.data(), n_ * sizeof(T), hipMemcpyHostToDevice, s), "upload");
    }
    void download(hipStream_t s = nullptr)
    {
        hip_throw(hipMemcpyAsync(host_.data(), dev_.data(), n_ * sizeof(T), hipMemcpyDeviceToHost, s), "download");
    }

private:
    size_t n_ = 0;
    PinnedArray<T> host_;
    DeviceArray<T> dev_;
};

}  // namespace qec
