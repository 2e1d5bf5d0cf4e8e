/*
 * CPU oracle in C (TEST INFRASTRUCTURE ONLY): a "cpu_ifirst-equivalent" restatement of the
 * four hot-path stencils of SURVEY.md §8(a), OpenMP over (K, J) rows, I innermost.
 *
 * Used only as (1) the full-size checker in the GPU parity tests and (2) bench.py's
 * cpu_baseline leg (kind "port"). Never linked into the gt4py_amd product path.
 *
 * Numerics follow the reference numpy backend op by op (compile with -ffp-contract=off):
 *   lap   = 4.0*u - (((u[i+1]+u[i-1])+u[j+1])+u[j-1])          stencil_definitions.py:316-320
 *   flx   = (res*(u[i+1]-u)) > 0 ? 0 : res, res = lap[i+1]-lap  stencil_definitions.py:321-322
 *   out   = u - coeff*(((flx-flx[i-1])+fly)-fly[j-1])           stencil_definitions.py:325-327
 *   f32   : lap/res/flx/fly in f64, neighbour sum in f32, out cast back to f32
 *           (gtir_upcaster.py:80-143; oracle-generated numpy module)
 *   tridiag: Thomas algorithm, stencil_definitions.py:219-232
 * Pinned by tests/test_oracle.py against the golden fixtures under tests/golden (reference numpy backend output).
 */
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <omp.h>

typedef struct {
    void* data;         /* element (0,0,0) of the array */
    int64_t stride[3];  /* elements */
    int64_t origin[3];
} ofield;

#define AT(f, T, i, j, k) \
    (((T*)(f)->data)[((f)->origin[0] + (i)) * (f)->stride[0] + ((f)->origin[1] + (j)) * (f)->stride[1] + \
                     ((f)->origin[2] + (k)) * (f)->stride[2]])

static void set_threads(int nthreads) {
    if (nthreads > 0) omp_set_num_threads(nthreads);
}

int oracle_copy_f64(const ofield* a, const ofield* b, int64_t ni, int64_t nj, int64_t nk, int nthreads) {
    set_threads(nthreads);
#pragma omp parallel for collapse(2) schedule(static)
    for (int64_t k = 0; k < nk; ++k)
        for (int64_t j = 0; j < nj; ++j)
            for (int64_t i = 0; i < ni; ++i) AT(b, double, i, j, k) = AT(a, double, i, j, k);
    return 0;
}

int oracle_lap5_f64(const ofield* u, const ofield* out, int64_t ni, int64_t nj, int64_t nk, int nthreads) {
    set_threads(nthreads);
#pragma omp parallel for collapse(2) schedule(static)
    for (int64_t k = 0; k < nk; ++k)
        for (int64_t j = 0; j < nj; ++j)
            for (int64_t i = 0; i < ni; ++i) {
                double s = ((AT(u, double, i + 1, j, k) + AT(u, double, i - 1, j, k)) + AT(u, double, i, j + 1, k)) +
                           AT(u, double, i, j - 1, k);
                AT(out, double, i, j, k) = 4.0 * AT(u, double, i, j, k) - s;
            }
    return 0;
}

/* lap at (i,j,k) computed in double; T is the field element type. */
#define HDIFF_IMPL(NAME, T)                                                                                \
    static inline double NAME##_lap(const ofield* u, int64_t i, int64_t j, int64_t k) {                    \
        T s = ((AT(u, T, i + 1, j, k) + AT(u, T, i - 1, j, k)) + AT(u, T, i, j + 1, k)) + AT(u, T, i, j - 1, k); \
        return 4.0 * (double)AT(u, T, i, j, k) - (double)s;                                                \
    }                                                                                                      \
    int oracle_##NAME(const ofield* u, const ofield* out, const ofield* coeff, int64_t ni, int64_t nj,     \
                      int64_t nk, int nthreads) {                                                          \
        set_threads(nthreads);                                                                             \
        _Pragma("omp parallel")                                                                            \
        {                                                                                                  \
            double* lm = (double*)malloc(sizeof(double) * (size_t)(ni + 2));                               \
            double* lc = (double*)malloc(sizeof(double) * (size_t)(ni + 2));                               \
            double* lp = (double*)malloc(sizeof(double) * (size_t)(ni + 2));                               \
            _Pragma("omp for collapse(2) schedule(static)")                                                \
            for (int64_t k = 0; k < nk; ++k)                                                               \
                for (int64_t j = 0; j < nj; ++j) {                                                         \
                    for (int64_t i = -1; i <= ni; ++i) {                                                   \
                        lc[i + 1] = NAME##_lap(u, i, j, k);                                                \
                        if (i >= 0 && i < ni) {                                                            \
                            lm[i + 1] = NAME##_lap(u, i, j - 1, k);                                        \
                            lp[i + 1] = NAME##_lap(u, i, j + 1, k);                                        \
                        }                                                                                  \
                    }                                                                                      \
                    for (int64_t i = 0; i < ni; ++i) {                                                     \
                        double r, flx, flxm, fly, flym;                                                    \
                        r = lc[i + 2] - lc[i + 1];                                                         \
                        flx = (r * (double)(AT(u, T, i + 1, j, k) - AT(u, T, i, j, k))) > 0.0 ? 0.0 : r;   \
                        r = lc[i + 1] - lc[i];                                                             \
                        flxm = (r * (double)(AT(u, T, i, j, k) - AT(u, T, i - 1, j, k))) > 0.0 ? 0.0 : r;  \
                        r = lp[i + 1] - lc[i + 1];                                                         \
                        fly = (r * (double)(AT(u, T, i, j + 1, k) - AT(u, T, i, j, k))) > 0.0 ? 0.0 : r;   \
                        r = lc[i + 1] - lm[i + 1];                                                         \
                        flym = (r * (double)(AT(u, T, i, j, k) - AT(u, T, i, j - 1, k))) > 0.0 ? 0.0 : r;  \
                        double res = (double)AT(u, T, i, j, k) -                                           \
                                     (double)AT(coeff, T, i, j, k) * (((flx - flxm) + fly) - flym);        \
                        AT(out, T, i, j, k) = (T)res;                                                      \
                    }                                                                                      \
                }                                                                                          \
            free(lm);                                                                                      \
            free(lc);                                                                                      \
            free(lp);                                                                                      \
        }                                                                                                  \
        return 0;                                                                                          \
    }

HDIFF_IMPL(hdiff_f64, double)
HDIFF_IMPL(hdiff_f32, float)

int oracle_tridiag_f64(const ofield* inf, const ofield* diag, const ofield* sup, const ofield* rhs, const ofield* out,
                       int64_t ni, int64_t nj, int64_t nk, int nthreads) {
    set_threads(nthreads);
#pragma omp parallel for schedule(static)
    for (int64_t j = 0; j < nj; ++j) {
        for (int64_t i = 0; i < ni; ++i) {
            AT(sup, double, i, j, 0) = AT(sup, double, i, j, 0) / AT(diag, double, i, j, 0);
            AT(rhs, double, i, j, 0) = AT(rhs, double, i, j, 0) / AT(diag, double, i, j, 0);
        }
        for (int64_t k = 1; k < nk; ++k)
            for (int64_t i = 0; i < ni; ++i) {
                double den = AT(diag, double, i, j, k) - AT(sup, double, i, j, k - 1) * AT(inf, double, i, j, k);
                AT(sup, double, i, j, k) = AT(sup, double, i, j, k) / den;
                AT(rhs, double, i, j, k) =
                    (AT(rhs, double, i, j, k) - AT(inf, double, i, j, k) * AT(rhs, double, i, j, k - 1)) / den;
            }
        for (int64_t i = 0; i < ni; ++i) AT(out, double, i, j, nk - 1) = AT(rhs, double, i, j, nk - 1);
        for (int64_t k = nk - 2; k >= 0; --k)
            for (int64_t i = 0; i < ni; ++i)
                AT(out, double, i, j, k) = AT(rhs, double, i, j, k) - AT(sup, double, i, j, k) * AT(out, double, i, j, k + 1);
    }
    return 0;
}
