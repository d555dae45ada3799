/*
 * oracle/tpe_score.c -- TEST INFRASTRUCTURE / CPU BASELINE ONLY.
 *
 * A plain-C restatement of the reference's candidate scoring, used as
 *   - the all-host-cores CPU baseline of bench.py (OpenMP over candidates),
 *   - a cross-check of the numpy oracle (tests/test_oracle.py).
 * It is never linked into the product library (hyperopt_amd/libhyperopt_tpe.so).
 *
 * Restated from mvanveen/hyperopt hyperopt/tpe.py:
 *   normal_cdf        :102-107     0.5 * (1 + erf((x - mu) / max(sqrt(2) sigma, EPS)))
 *   GMM1_lpdf         :110-172     q None: logsum_rows(-0.5 mahal^2 + log(w / Z / p_accept))
 *                                  q:      log(sum_k w Phi(ub) - w Phi(lb)) - log(p_accept)
 *   lognormal_cdf     :177-196     .5 + .5 erf((log(max(x, EPS)) - mu) / max(sqrt(2) sigma, EPS))
 *   lognormal_lpdf    :199-208     -E - log(sigma x sqrt(2 pi)), sigma = max(sigma, EPS)
 *   logsum_rows       :259-262     two-pass: row max, then log(sum exp(x - max)) + max
 *   LGMM1_lpdf        :265-307     (q None ignores p_accept -- reference quirk)
 *   categorical_lpdf  :56-63       log(p[sample])
 *   broadcast_best    :769-778     np.argmax(below - above): first NaN, else first max
 * p_accept is summed sequentially here (numpy sums pairwise); the difference is
 * a few ulp and the numpy oracle, not this file, pins bit-level parity.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

#define EPS 1e-12
#define HAS_LOW 1
#define HAS_HIGH 2
#define HAS_Q 4

static double normal_cdf(double x, double mu, double sigma) {
    double bottom = fmax(sqrt(2.0) * sigma, EPS);
    return 0.5 * (1.0 + erf((x - mu) / bottom));
}

static double lognormal_cdf(double x, double mu, double sigma) {
    double top = log(fmax(x, EPS)) - mu;
    double bottom = fmax(sqrt(2.0) * sigma, EPS);
    return .5 + .5 * erf(top / bottom);
}

double ora_p_accept(const double *w, const double *mu, const double *s, int k, int flags,
                    double low, double high) {
    if ((flags & (HAS_LOW | HAS_HIGH)) == 0) return 1.0;
    double p = 0.0;
    for (int j = 0; j < k; ++j) p += w[j] * (normal_cdf(high, mu[j], s[j]) - normal_cdf(low, mu[j], s[j]));
    return p;
}

/* GMM1_lpdf (log_space = 0) / LGMM1_lpdf (log_space = 1) of n samples */
void ora_mixture_lpdf(int log_space, const double *x, int64_t n, const double *w, const double *mu,
                      const double *s, int k, int flags, double low, double high, double q,
                      double *out) {
    const double p_accept = ora_p_accept(w, mu, s, k, flags, low, high);
    const double lpacc = log(p_accept);
    const double SQ2PI = sqrt(2.0 * M_PI);
    if (!(flags & HAS_Q)) {
        /* per-component constants, as numpy forms them once per call:
         * GMM1 log(w / sqrt(2 pi sigma^2) / p_accept), LGMM1 log(w) */
        double *lc = (double *)malloc(sizeof(double) * (k > 0 ? k : 1));
        for (int j = 0; j < k; ++j)
            lc[j] = log_space ? log(w[j]) : log(w[j] / sqrt(2.0 * M_PI * (s[j] * s[j])) / p_accept);
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < n; ++i) {
            const double xi = x[i];
            const double lx = log_space ? log(xi) : 0.0;
            double m = -INFINITY;
            for (int pass = 0; pass < 2; ++pass) {
                double acc = 0.0;
                for (int j = 0; j < k; ++j) {
                    double t;
                    if (!log_space) {
                        const double d = (xi - mu[j]) / fmax(s[j], EPS);
                        t = -0.5 * (d * d) + lc[j];
                    } else {
                        const double sg = fmax(s[j], EPS);
                        const double e = (lx - mu[j]) / sg;
                        t = (-(0.5 * (e * e)) - log(sg * xi * SQ2PI)) + lc[j];
                    }
                    if (pass == 0) {
                        if (m == m && (t != t || t > m)) m = t;   /* np.max: NaN propagates */
                    } else {
                        acc += exp(t - m);
                    }
                }
                if (pass == 1) out[i] = log(acc) + m;
            }
        }
        free(lc);
        return;
    }
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        const double xi = x[i];
        double ub = xi + q / 2.0, lb = xi - q / 2.0;
        if (!log_space) {
            if (flags & HAS_HIGH) ub = fmin(ub, high);
            if (flags & HAS_LOW) lb = fmax(lb, low);
        } else {
            if (flags & HAS_HIGH) ub = fmin(ub, exp(high));
            if (flags & HAS_LOW) lb = fmax(lb, exp(low));
            lb = fmax(0.0, lb);
        }
        double prob = 0.0;
        for (int j = 0; j < k; ++j) {
            double inc, pl;
            if (!log_space) {
                inc = w[j] * normal_cdf(ub, mu[j], s[j]);
                pl = w[j] * normal_cdf(lb, mu[j], s[j]);
            } else {
                inc = w[j] * lognormal_cdf(ub, mu[j], s[j]);
                pl = w[j] * lognormal_cdf(lb, mu[j], s[j]);
            }
            inc -= pl;
            prob += inc;
        }
        out[i] = log(prob) - lpacc;
    }
}

void ora_categorical_lpdf(const int64_t *sample, int64_t n, const double *p, double *out) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) out[i] = log(p[sample[i]]);
}

int64_t ora_broadcast_best(const double *below, const double *above, int64_t n) {
    int64_t best = 0;
    double bs = -INFINITY;
    for (int64_t i = 0; i < n; ++i) {
        const double sc = below[i] - above[i];
        if (sc != sc) return i;            /* first NaN wins */
        if (i == 0 || sc > bs) {
            bs = sc;
            best = i;
        }
    }
    return best;
}

int ora_threads(void) {
#ifdef _OPENMP
    extern int omp_get_max_threads(void);
    return omp_get_max_threads();
#else
    return 1;
#endif
}
