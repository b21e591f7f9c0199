/**
 * @file device.cpp
 * HIP runtime calls behind blf/device.h (allocation, copies, the per-thread handle).
 */
#include <hip/hip_runtime_api.h>

#include <blf/device.h>

namespace blf
{

namespace
{
struct HandleHolder
{
    blf_handle* h{nullptr};
    bool tried{false};
    ~HandleHolder()
    {
        if (h != nullptr) blf_destroy(h);
    }
};
thread_local HandleHolder t_handle;
} // namespace

blf_handle* threadHandle()
{
    if (!t_handle.tried)
    {
        t_handle.tried = true;
        if (blf_create(&t_handle.h, 0) != BLF_OK)
        {
            std::cerr << "[blf::threadHandle] " << blf_last_error() << std::endl;
            t_handle.h = nullptr;
        }
    }
    return t_handle.h;
}

bool report(blf_status status, const char* where)
{
    if (status == BLF_OK) return true;
    std::cerr << "[" << where << "] " << blf_last_error() << std::endl;
    return false;
}

bool synchronize()
{
    return hipDeviceSynchronize() == hipSuccess;
}

bool copyRows(void* dst, std::size_t dpitch, const void* src, std::size_t spitch,
              std::size_t width, std::size_t rows)
{
    if (rows == 0) return true;
    if (hipMemcpy2DAsync(dst, dpitch, src, spitch, width, rows, hipMemcpyDeviceToDevice,
                         nullptr) != hipSuccess)
    {
        std::cerr << "[blf::copyRows] hipMemcpy2DAsync failed" << std::endl;
        return false;
    }
    return true;
}

template <typename T> void* DeviceBuffer<T>::alloc(std::size_t bytes)
{
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess)
    {
        std::cerr << "[blf::DeviceBuffer] hipMalloc of " << bytes << " bytes failed" << std::endl;
        return nullptr;
    }
    return p;
}

template <typename T> void DeviceBuffer<T>::release(void* p)
{
    if (p != nullptr) (void)hipFree(p);
}

template <typename T> bool DeviceBuffer<T>::copy(void* dst, const void* src, std::size_t bytes, int kind)
{
    const hipMemcpyKind k = kind == 1 ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost;
    if (hipMemcpy(dst, src, bytes, k) != hipSuccess)
    {
        std::cerr << "[blf::DeviceBuffer] hipMemcpy failed" << std::endl;
        return false;
    }
    return true;
}

template class DeviceBuffer<double>;
template class DeviceBuffer<int32_t>;

} // namespace blf
