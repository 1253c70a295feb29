/* ptrattr.hip -- development probe: what hipPointerGetAttributes reports
 * for interior pointers of hipHostMalloc / hipHostRegister memory. */
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

static void show(const char *what, void *p)
{
    hipPointerAttribute_t a;
    hipError_t e = hipPointerGetAttributes(&a, p);
    void *dp = nullptr;
    hipError_t e2 = hipHostGetDevicePointer(&dp, p, 0);
    printf("%-22s p=%p rc=%d type=%d host=%p dev=%p | getDevPtr rc=%d dp=%p\n", what, p, (int)e,
           (int)a.type, a.hostPointer, a.devicePointer, (int)e2, dp);
    (void)hipGetLastError();
}

int main()
{
    void *h;
    if (hipHostMalloc(&h, 1 << 24, hipHostMallocDefault) != hipSuccess)
        return 1;
    show("hostmalloc base", h);
    show("hostmalloc +4096+5", (char *)h + 4101);
    void *m = aligned_alloc(4096, 1 << 24);
    show("malloc (unregistered)", m);
    if (hipHostRegister(m, 1 << 24, hipHostRegisterDefault) != hipSuccess)
        printf("register failed\n");
    show("registered base", m);
    show("registered +8192+3", (char *)m + 8195);
    void *m2 = malloc((1 << 24) + 100);
    if (hipHostRegister((char *)m2 + 100, 1 << 24, hipHostRegisterMapped) != hipSuccess)
        printf("register2 failed\n");
    show("registered unaligned", (char *)m2 + 100);
    show("registered unal. +77", (char *)m2 + 177);
    return 0;
}
