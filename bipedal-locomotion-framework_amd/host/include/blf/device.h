/**
 * @file device.h
 * Host-side plumbing of the C++ adapters: RAII device buffers and a per-thread blf_handle.
 * Every compute call of the adapters goes through include/blf/blf_c.h (the HIP kernels); if no
 * HIP device is present the adapters report the failure in the reference's style (false + a
 * "[Class::method]" line on std::cerr) — there is no CPU fallback.
 */
#ifndef BLF_HOST_DEVICE_H
#define BLF_HOST_DEVICE_H

#include <cstddef>
#include <cstdint>
#include <iostream>
#include <string>
#include <vector>

#include <blf/blf_c.h>

namespace blf
{

/** The calling thread's library handle (device 0), created on first use; nullptr on failure. */
blf_handle* threadHandle();

/** Print "[where] <library error>" on std::cerr if status != BLF_OK; returns status == BLF_OK. */
bool report(blf_status status, const char* where);

/** Owning device allocation of n elements of T (hipMalloc / hipFree). */
template <typename T> class DeviceBuffer
{
    void* m_ptr{nullptr};
    std::size_t m_size{0};

    static void* alloc(std::size_t bytes);
    static void release(void* p);
    static bool copy(void* dst, const void* src, std::size_t bytes, int kind);

public:
    DeviceBuffer() = default;
    explicit DeviceBuffer(std::size_t n) { resize(n); }
    DeviceBuffer(const DeviceBuffer&) = delete;
    DeviceBuffer& operator=(const DeviceBuffer&) = delete;
    DeviceBuffer(DeviceBuffer&& o) noexcept : m_ptr(o.m_ptr), m_size(o.m_size)
    {
        o.m_ptr = nullptr;
        o.m_size = 0;
    }
    ~DeviceBuffer() { release(m_ptr); }

    /** Reallocate if the size changes (contents are not preserved). */
    bool resize(std::size_t n)
    {
        if (n == m_size && (m_ptr != nullptr || n == 0)) return true;
        release(m_ptr);
        m_ptr = nullptr;
        m_size = 0;
        if (n == 0) return true;
        m_ptr = alloc(n * sizeof(T));
        if (m_ptr == nullptr) return false;
        m_size = n;
        return true;
    }
    T* data() { return static_cast<T*>(m_ptr); }
    const T* data() const { return static_cast<const T*>(m_ptr); }
    std::size_t size() const { return m_size; }

    bool upload(const T* host, std::size_t n)
    {
        return resize(n) && (n == 0 || copy(m_ptr, host, n * sizeof(T), 1));
    }
    bool upload(const std::vector<T>& host) { return upload(host.data(), host.size()); }
    bool download(T* host, std::size_t n) const
    {
        return n <= m_size && (n == 0 || copy(host, m_ptr, n * sizeof(T), 2));
    }
    bool download(std::vector<T>& host) const
    {
        host.resize(m_size);
        return download(host.data(), m_size);
    }
};

/** Waits for all work queued by this thread on the default stream. */
bool synchronize();

/** Stream-ordered device-to-device copy of `rows` rows of `width` bytes between pitched
 * layouts (hipMemcpy2DAsync on the default stream). */
bool copyRows(void* dst, std::size_t dpitch, const void* src, std::size_t spitch,
              std::size_t width, std::size_t rows);

} // namespace blf

#endif // BLF_HOST_DEVICE_H
