/* C restatement of the reference mixing path -- TEST INFRASTRUCTURE ONLY.
 *
 * Restates utils/consensus_simple/mixer.py:43-49 (Mixer._mix_params_once) and
 * mixer.py:57-66 (_get_deviation_dict: np.mean over agents, then ||x_a - mean||) in plain C.
 * Built with -ffp-contract=off so every product and sum rounds separately, as numpy does;
 * tests/test_oracle_golden.py checks it bit-exact against the reference-generated fixtures.
 * Used by the tests as a fast checker at mid sizes and by bench.py as the timed CPU baseline
 * ("port", single thread).  Never linked into the product library.
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

/* out[a, :] = sum_{e in row a} w[e] * x[col[e], :]  (left fold starting at +0.0).
 * Optional fused local step: x <- x - lr * g applied to every source row first
 * (g == NULL: plain mix).  Column-blocked so each source row block stays in cache. */
void ref_mix_round(const float *x, int64_t ldx, const float *g, int64_t ldg, float lr,
                   float *out, int64_t ldo, int32_t n_rows, int64_t n_params,
                   const int64_t *rowptr, const int64_t *col, const double *w,
                   float *scratch /* n_rows*block floats when g != NULL */, int64_t block) {
    for (int64_t p0 = 0; p0 < n_params; p0 += block) {
        int64_t pb = n_params - p0 < block ? n_params - p0 : block;
        const float *src = x + p0;
        int64_t lds = ldx;
        if (g) {
            for (int32_t r = 0; r < n_rows; ++r)
                for (int64_t p = 0; p < pb; ++p) {
                    float t = lr * g[r * ldg + p0 + p];
                    scratch[r * block + p] = x[r * ldx + p0 + p] - t;
                }
            src = scratch;
            lds = block;
        }
        for (int32_t a = 0; a < n_rows; ++a) {
            float *o = out + a * ldo + p0;
            for (int64_t p = 0; p < pb; ++p) o[p] = 0.0f;
            for (int64_t e = rowptr[a]; e < rowptr[a + 1]; ++e) {
                const float we = (float)w[e];
                const float *s = src + col[e] * lds;
                for (int64_t p = 0; p < pb; ++p) {
                    float prod = s[p] * we;
                    o[p] = o[p] + prod;
                }
            }
        }
    }
}

/* mean[p] = (sum_r x[r,p]) / n_rows, rows added in order (numpy add.reduce over axis 0). */
void ref_column_mean(const float *x, int64_t ldx, int32_t n_rows, int64_t n_params, float *mean) {
    memcpy(mean, x, (size_t)n_params * sizeof(float));
    for (int32_t r = 1; r < n_rows; ++r)
        for (int64_t p = 0; p < n_params; ++p) mean[p] = mean[p] + x[r * ldx + p];
    const float n = (float)n_rows;
    for (int64_t p = 0; p < n_params; ++p) mean[p] = mean[p] / n;
}

/* dev_sq[a] = sum_p (x[a,p] - mean[p])^2, accumulated in double (the reference's fp32 BLAS
 * dot order is not reproducible; parity for this value is a tolerance, not bit-exact). */
void ref_deviation_sq(const float *x, int64_t ldx, int32_t n_rows, int64_t n_params,
                      const float *mean, double *dev_sq) {
    for (int32_t a = 0; a < n_rows; ++a) {
        double s = 0.0;
        for (int64_t p = 0; p < n_params; ++p) {
            float d = x[a * ldx + p] - mean[p];
            s += (double)d * (double)d;
        }
        dev_sq[a] = s;
    }
}

/* torch.optim.SGD.step (torch/optim/sgd.py, single-tensor form) on an [n_rows, n_params] block,
 * restated with explicit fmaf for each of torch's add-with-alpha (ATen's add kernels compute
 * a + alpha*b as one fused multiply-add) -- the local step of config c5 (Man_Colab.ipynb cell 19).
 *   d = g + wd*x;  buf = first ? d : mu*buf + (1-damp)*d;  d = nesterov ? d + mu*buf : buf;
 *   out = x - lr*d      (buf may be NULL when mu == 0; out may alias x) */
void ref_sgd_step(const float *x, int64_t ldx, const float *g, int64_t ldg, float *buf,
                  int64_t ldb, float *out, int64_t ldo, int32_t n_rows, int64_t n_params,
                  float lr, float mu, float damp, float wd, int32_t nesterov, int32_t first) {
    for (int32_t r = 0; r < n_rows; ++r)
        for (int64_t p = 0; p < n_params; ++p) {
            const float xv = x[r * ldx + p];
            float d = g[r * ldg + p];
            if (wd != 0.0f) d = fmaf(wd, xv, d);
            if (mu != 0.0f) {
                float *b = buf + r * ldb + p;
                if (first) {
                    *b = d;
                } else {
                    const float m = mu * *b;
                    *b = fmaf(1.0f - damp, d, m);
                }
                d = nesterov ? fmaf(mu, *b, d) : *b;
            }
            out[r * ldo + p] = fmaf(-lr, d, xv);
        }
}
