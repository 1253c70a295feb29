/*
 * ec_jitc.c -- the compiler process of the run-time compiled kernels
 * (ec_jit.hip, r06).
 *
 *   ec_jitc SOURCE CODE_OBJECT
 *
 * Compiles one generated kernel source for gfx950 with hiprtc and writes the
 * code object; the compiler's messages go to stderr.  Exit status 0 on
 * success, 1 when the compiler failed, 2 without hiprtc, 3 on I/O errors.
 *
 * The library runs this as a child process instead of calling hiprtc in the
 * client: LLVM then never lives in a GlusterFS client's address space, and a
 * client that exits while a compile is running is not taken down by the
 * compiler's static destructors running under a compile in another thread
 * (which crashed every such exit when the compile ran on a library thread).
 */
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef int (*create_t)(void **, const char *, const char *, int, const char *const *,
                        const char *const *);
typedef int (*compile_t)(void *, int, const char *const *);
typedef int (*size_fn)(void *, size_t *);
typedef int (*get_t)(void *, char *);
typedef int (*destroy_t)(void **);

static char *slurp(const char *path, size_t *n)
{
    FILE *f = fopen(path, "rb");
    char *b = NULL;
    long len;

    if (!f)
        return NULL;
    if (fseek(f, 0, SEEK_END) == 0 && (len = ftell(f)) >= 0 && fseek(f, 0, SEEK_SET) == 0 &&
        (b = malloc((size_t)len + 1)) != NULL) {
        *n = fread(b, 1, (size_t)len, f);
        b[*n] = 0;
    }
    fclose(f);
    return b;
}

int main(int argc, char **argv)
{
    static const char *libs[] = {"libhiprtc.so.7", "libhiprtc.so", "/opt/rocm/lib/libhiprtc.so.7"};
    const char *opts[] = {"--offload-arch=gfx950", "-O3"};
    void *h = NULL, *prog = NULL;
    size_t n = 0, cs = 0, ls = 0;
    char *src, *code, *log;
    FILE *o;
    int rc;

    if (argc != 3) {
        fprintf(stderr, "usage: %s SOURCE CODE_OBJECT\n", argv[0]);
        return 3;
    }
    for (size_t i = 0; i < sizeof(libs) / sizeof(libs[0]) && !h; i++)
        h = dlopen(libs[i], RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        fprintf(stderr, "ec_jitc: libhiprtc not found\n");
        return 2;
    }
    create_t create = (create_t)dlsym(h, "hiprtcCreateProgram");
    compile_t compile = (compile_t)dlsym(h, "hiprtcCompileProgram");
    size_fn log_size = (size_fn)dlsym(h, "hiprtcGetProgramLogSize");
    get_t get_log = (get_t)dlsym(h, "hiprtcGetProgramLog");
    size_fn code_size = (size_fn)dlsym(h, "hiprtcGetCodeSize");
    get_t get_code = (get_t)dlsym(h, "hiprtcGetCode");
    destroy_t destroy = (destroy_t)dlsym(h, "hiprtcDestroyProgram");
    if (!create || !compile || !log_size || !get_log || !code_size || !get_code || !destroy) {
        fprintf(stderr, "ec_jitc: libhiprtc lacks an entry point\n");
        return 2;
    }
    if (!(src = slurp(argv[1], &n))) {
        fprintf(stderr, "ec_jitc: cannot read %s\n", argv[1]);
        return 3;
    }
    if (create(&prog, src, "ec_jit.hip", 0, NULL, NULL) != 0) {
        fprintf(stderr, "ec_jitc: hiprtcCreateProgram failed\n");
        return 1;
    }
    rc = compile(prog, 2, opts);
    if (log_size(prog, &ls) == 0 && ls > 1 && (log = malloc(ls)) != NULL) {
        if (get_log(prog, log) == 0)
            fwrite(log, 1, strlen(log), stderr);
        free(log);
    }
    if (rc != 0 || code_size(prog, &cs) != 0 || cs == 0 || !(code = malloc(cs)) ||
        get_code(prog, code) != 0) {
        fprintf(stderr, "ec_jitc: compilation failed (%d)\n", rc);
        return 1;
    }
    if (!(o = fopen(argv[2], "wb")) || fwrite(code, 1, cs, o) != cs || fclose(o) != 0) {
        fprintf(stderr, "ec_jitc: cannot write %s\n", argv[2]);
        return 3;
    }
    destroy(&prog);
    return 0;
}
