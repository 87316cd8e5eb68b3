/* Test helper (tests/test_teardown.py): interposes the HIP entry points that
 * liblvgpu.so calls, counts the calls made from liblvgpu.so, and reports the
 * ones made after the test armed it at interpreter exit -- i.e. from the
 * library's static destructors (__cxa_finalize), which run after Python's
 * atexit hooks and before this file's exit handler (registered first, so it
 * runs last).  Each wrapper forwards to the runtime the library binds to
 * (torch's, loaded first), or reports hipErrorNotInitialized without one. */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int g_armed = 0;
static long g_calls = 0, g_late = 0;
static char g_late_names[512];

static int from_lvgpu(void *ra) {
    Dl_info di;
    return dladdr(ra, &di) && di.dli_fname && strstr(di.dli_fname, "liblvgpu") != NULL;
}

static void note(const char *name, void *ra) {
    if (!from_lvgpu(ra)) return;
    ++g_calls;
    if (g_armed) {
        ++g_late;
        if (strlen(g_late_names) + strlen(name) + 2 < sizeof g_late_names) {
            strcat(g_late_names, name);
            strcat(g_late_names, " ");
        }
    }
}

static void report(void) {
    fprintf(stderr, "hipspy: calls_from_lvgpu=%ld calls_after_exit=%ld [%s]\n", g_calls, g_late, g_late_names);
}

__attribute__((constructor)) static void init(void) { atexit(report); }

void hipspy_arm(void) { g_armed = 1; }
long hipspy_calls(void) { return g_calls; }

/* The runtime liblvgpu.so itself binds to (torch's copy, already loaded
 * under the libamdhip64 soname), else the next definition. */
static void *sym(const char *name) {
    static void *rt = NULL;
    if (!rt) rt = dlopen("libamdhip64.so.7", RTLD_NOLOAD | RTLD_NOW);
    if (!rt) rt = dlopen("libamdhip64.so", RTLD_NOLOAD | RTLD_NOW);
    void *f = rt ? dlsym(rt, name) : NULL;
    return f ? f : dlsym(RTLD_NEXT, name);
}

typedef int (*fn1)(void *);
typedef int (*fn2)(void *, size_t);
typedef int (*fn3)(void **, size_t, unsigned);

#define FWD1(name)                                                      \
    int name(void *p) {                                                 \
        note(#name, __builtin_return_address(0));                       \
        fn1 f = (fn1)sym(#name);                           \
        return f ? f(p) : 3; /* hipErrorNotInitialized */               \
    }
FWD1(hipFree)
FWD1(hipHostFree)
FWD1(hipStreamDestroy)
FWD1(hipEventDestroy)
FWD1(hipStreamSynchronize)
FWD1(hipEventSynchronize)

int hipMalloc(void **p, size_t n) {
    note("hipMalloc", __builtin_return_address(0));
    fn2 f = (fn2)sym("hipMalloc");
    return f ? ((int (*)(void **, size_t))f)(p, n) : 3;
}

int hipHostMalloc(void **p, size_t n, unsigned flags) {
    note("hipHostMalloc", __builtin_return_address(0));
    fn3 f = (fn3)sym("hipHostMalloc");
    return f ? f(p, n, flags) : 3;
}
