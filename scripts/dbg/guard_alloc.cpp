// Debug allocator for torch.cuda.memory.CUDAPluggableAllocator: every allocation is padded by
// guard regions on both sides and the whole block (guards and payload) is filled with 0xFF
// bytes (float NaN, int -1): a kernel that reads outside its tensors or reads memory no kernel
// wrote sees NaN, and a kernel that writes outside its tensors is reported when the block is
// freed (size, side, offset of the first changed guard byte).  Test tooling only.
#include <hip/hip_runtime.h>
#include <sys/types.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

static const size_t G = 64 << 10;
static long long g_seq = 0;

extern "C" void* guard_alloc(ssize_t size, int device, hipStream_t stream) {
    (void)device;
    void* base = nullptr;
    const size_t pay = ((size_t)size + 255) / 256 * 256;
    const size_t tot = pay + 2 * G + 256;
    if (hipMalloc(&base, tot) != hipSuccess) return nullptr;
    (void)hipMemsetAsync(base, 0xFF, tot, stream);
    (void)hipStreamSynchronize(stream);
    // header: payload size and sequence number, in the first 16 bytes of the front guard
    long long hdr[2] = {(long long)size, g_seq++};
    (void)hipMemcpy(base, hdr, sizeof(hdr), hipMemcpyHostToDevice);
    return (char*)base + 256 + G;
}

extern "C" void guard_free(void* ptr, ssize_t size, int device, hipStream_t stream) {
    (void)device; (void)stream;
    (void)hipDeviceSynchronize();
    char* base = (char*)ptr - G - 256;
    const size_t pay = ((size_t)size + 255) / 256 * 256;
    std::vector<unsigned char> front(G), back(G + (pay - (size_t)size));
    (void)hipMemcpy(front.data(), base + 256, G, hipMemcpyDeviceToHost);
    (void)hipMemcpy(back.data(), (char*)ptr + size, back.size(), hipMemcpyDeviceToHost);
    long long hdr[2];
    (void)hipMemcpy(hdr, base, sizeof(hdr), hipMemcpyDeviceToHost);
    for (size_t i = 0; i < G; ++i)
        if (front[i] != 0xFF) {
            fprintf(stderr, "GUARD front written: alloc #%lld size %zd, %zu bytes before the start\n", hdr[1],
                    size, G - i);
            break;
        }
    for (size_t i = 0; i < back.size(); ++i)
        if (back[i] != 0xFF) {
            fprintf(stderr, "GUARD back written: alloc #%lld size %zd, byte %zu past the end\n", hdr[1], size, i);
            break;
        }
    (void)hipFree(base);
}
