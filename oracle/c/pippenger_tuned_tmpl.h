/* Tuned CPU batch combination -- TEST / BASELINE INFRASTRUCTURE ONLY (like the rest of oracle/).
 *
 * Loaded only by tests/ (checked against the plain oracle above it, bit for bit) and by
 * bench.py's cpu_baseline leg, where it is the "competent CPU verifier" the GPU rate is quoted
 * against.  Never by the product package.
 *
 * Include-template after curve_tmpl.h (same macros).  Computes the same A = sum r_i pi_i and
 * B = sum r_i C_i + s_i pi_i - t G1 as C_(batch_verify) (same randomisers, same SRS G1), with
 * the textbook performance techniques of CPU Pippenger implementations -- restated here, not
 * taken from any library:
 *   - signed window digits (|d| <= 2^(c-1): half the buckets), recoded once per scalar;
 *   - XYZZ bucket coordinates with the mixed addition madd-2008-s (8M + 2S per term) and
 *     add-2008-s / dbl-2008-s-1 for the bucket-sum reduction (EFD formulas for
 *     short-Weierstrass a = 0);
 *   - the two MSMs fused into one term list (MSM#0 over pi with r, MSM#1 over C with r, pi
 *     with s and G1 with -t), the 127-bit r_i using only the low windows;
 *   - a CIOS Montgomery product on 64-bit limbs with mulx/adcx/adox (two interleaved carry
 *     chains, tmul_x86_gen.h from oracle/gen_tmul_x86.py; an unsigned __int128 form elsewhere),
 *     lazy by one subtraction because the moduli leave a spare top bit (p < 2^381 / 2^254);
 *   - OpenMP over (MSM, window, point-range) tasks with dynamic scheduling, one bucket array
 *     per task (c = 13 keeps 4096 x 192 B of buckets in a core's L2).
 * The pairing check (C_(pairing_check_fast), below) uses the same Miller loop as the oracle
 * with its line functions precomputed once per SRS G2 pair (the T sequence depends only on Q),
 * and a final exponentiation split into the easy part (conjugate / inverse / Frobenius^2) and
 * the hard part as a 4-term Frobenius multi-exponent with Granger-Scott cyclotomic squarings
 * (fexp_gen.h, oracle/gen_fexp.py) -- the same value as the oracle's plain-pow exponentiation.
 * Reference: none (/root/reference/LICENSE:1-201 only).
 */
typedef struct { FP x, y, zz, zzz; } C_(xyzz);  /* x = X/ZZ, y = Y/ZZZ (ZZ^3 = ZZZ^2); ZZ = 0 <=> O */
static void C_(pairing_check_fast)(const C_(aff)* A, const C_(aff)* B, const C_(aff2)* g2, const C_(aff2)* tg2,
                                   int* ok);

/* Montgomery product (a b) / 2^(64 FN) mod p, result < p.  x86-64 with BMI2 + ADX: the
 * generated mulx/adcx/adox CIOS (tmul_x86_gen.h, two interleaved carry chains); otherwise a
 * no-carry CIOS on unsigned __int128, fully unrolled.  Both leave t < 2p (spare top bit of p). */
static inline __attribute__((always_inline)) void C_(tmul)(FP* r, const FP* a, const FP* b) {
  enum { N = (int)(sizeof(FP) / 8) };
  uint64_t t[N];
#if defined(__x86_64__) && defined(__ADX__) && defined(__BMI2__) && !defined(KZGO_NO_ASM)
  if (N == 6) tmul_x86_6(t, a->v, b->v, PRAW, PINV_T);
  else tmul_x86_4(t, a->v, b->v, PRAW, PINV_T);
#else
  uint64_t av[N];
#pragma GCC unroll 8
  for (int j = 0; j < N; ++j) { t[j] = 0; av[j] = a->v[j]; }
#pragma GCC unroll 8
  for (int i = 0; i < N; ++i) {
    const uint64_t bi = b->v[i];
    unsigned __int128 A = (unsigned __int128)av[0] * bi + t[0];
    const uint64_t t0 = (uint64_t)A;
    uint64_t ca = (uint64_t)(A >> 64);
    const uint64_t m = t0 * PINV_T;
    unsigned __int128 Cc = (unsigned __int128)m * PRAW[0] + t0;
    uint64_t cc = (uint64_t)(Cc >> 64);
#pragma GCC unroll 8
    for (int j = 1; j < N; ++j) {
      A = (unsigned __int128)av[j] * bi + t[j] + ca;
      ca = (uint64_t)(A >> 64);
      Cc = (unsigned __int128)m * PRAW[j] + (uint64_t)A + cc;
      t[j - 1] = (uint64_t)Cc;
      cc = (uint64_t)(Cc >> 64);
    }
    t[N - 1] = cc + ca;
  }
#endif
  /* t < 2p: one conditional subtraction */
  uint64_t d[N], bw = 0;
#pragma GCC unroll 8
  for (int j = 0; j < N; ++j) {
    const unsigned __int128 x = (unsigned __int128)t[j] - PRAW[j] - bw;
    d[j] = (uint64_t)x;
    bw = (uint64_t)(x >> 64) & 1;
  }
  const uint64_t keep = 0 - bw;  /* borrow: t < p, keep t */
#pragma GCC unroll 8
  for (int j = 0; j < N; ++j) r->v[j] = (t[j] & keep) | (d[j] & ~keep);
}
static inline void C_(tsqr)(FP* r, const FP* a) { C_(tmul)(r, a, a); }

static inline void C_(xyzz_set_inf)(C_(xyzz)* p) {
  FP_(one)(&p->x); FP_(one)(&p->y); FP_(zero)(&p->zz); FP_(zero)(&p->zzz);
}
static inline int C_(xyzz_is_inf)(const C_(xyzz)* p) { return FP_(is_zero)(&p->zz); }

/* p = 2 q for affine q (mdbl-2008-s-1) */
static void C_(xyzz_dbl_aff)(C_(xyzz)* p, const FP* qx, const FP* qy) {
  FP U, V, W, S, M, t;
  FP_(dbl)(&U, qy);
  C_(tsqr)(&V, &U);
  C_(tmul)(&W, &U, &V);
  C_(tmul)(&S, qx, &V);
  C_(tsqr)(&t, qx); FP_(dbl)(&M, &t); FP_(add)(&M, &M, &t);
  C_(tsqr)(&p->x, &M); FP_(dbl)(&t, &S); FP_(sub)(&p->x, &p->x, &t);
  FP_(sub)(&t, &S, &p->x); C_(tmul)(&p->y, &M, &t);
  C_(tmul)(&t, &W, qy); FP_(sub)(&p->y, &p->y, &t);
  p->zz = V; p->zzz = W;
}

/* p = 2 p (dbl-2008-s-1, a = 0) */
static void C_(xyzz_dbl)(C_(xyzz)* p) {
  if (C_(xyzz_is_inf)(p)) return;
  FP U, V, W, S, M, t, x3;
  FP_(dbl)(&U, &p->y);
  C_(tsqr)(&V, &U);
  C_(tmul)(&W, &U, &V);
  C_(tmul)(&S, &p->x, &V);
  C_(tsqr)(&t, &p->x); FP_(dbl)(&M, &t); FP_(add)(&M, &M, &t);
  C_(tsqr)(&x3, &M); FP_(dbl)(&t, &S); FP_(sub)(&x3, &x3, &t);
  FP_(sub)(&t, &S, &x3); C_(tmul)(&t, &M, &t);
  FP y3; C_(tmul)(&y3, &W, &p->y); FP_(sub)(&y3, &t, &y3);
  C_(tmul)(&p->zz, &p->zz, &V); C_(tmul)(&p->zzz, &p->zzz, &W);
  p->x = x3; p->y = y3;
}

/* p += (qx, qy) affine, not infinity (madd-2008-s: 8M + 2S) */
static void C_(xyzz_madd)(C_(xyzz)* p, const FP* qx, const FP* qy) {
  if (C_(xyzz_is_inf)(p)) {
    p->x = *qx; p->y = *qy; FP_(one)(&p->zz); FP_(one)(&p->zzz);
    return;
  }
  FP U2, S2, P, R, PP, PPP, Q, t;
  C_(tmul)(&U2, qx, &p->zz);
  C_(tmul)(&S2, qy, &p->zzz);
  FP_(sub)(&P, &U2, &p->x);
  FP_(sub)(&R, &S2, &p->y);
  if (FP_(is_zero)(&P)) {
    if (FP_(is_zero)(&R)) C_(xyzz_dbl_aff)(p, qx, qy);
    else C_(xyzz_set_inf)(p);
    return;
  }
  C_(tsqr)(&PP, &P);
  C_(tmul)(&PPP, &P, &PP);
  C_(tmul)(&Q, &p->x, &PP);
  FP x3; C_(tsqr)(&x3, &R); FP_(sub)(&x3, &x3, &PPP); FP_(dbl)(&t, &Q); FP_(sub)(&x3, &x3, &t);
  FP_(sub)(&t, &Q, &x3); C_(tmul)(&t, &R, &t);
  FP y3; C_(tmul)(&y3, &p->y, &PPP); FP_(sub)(&p->y, &t, &y3);
  p->x = x3;
  C_(tmul)(&p->zz, &p->zz, &PP);
  C_(tmul)(&p->zzz, &p->zzz, &PPP);
}

/* p += q, both XYZZ (add-2008-s) */
static void C_(xyzz_add)(C_(xyzz)* p, const C_(xyzz)* q) {
  if (C_(xyzz_is_inf)(q)) return;
  if (C_(xyzz_is_inf)(p)) { *p = *q; return; }
  FP U1, U2, S1, S2, P, R, PP, PPP, Q, t;
  C_(tmul)(&U1, &p->x, &q->zz);
  C_(tmul)(&U2, &q->x, &p->zz);
  C_(tmul)(&S1, &p->y, &q->zzz);
  C_(tmul)(&S2, &q->y, &p->zzz);
  FP_(sub)(&P, &U2, &U1);
  FP_(sub)(&R, &S2, &S1);
  if (FP_(is_zero)(&P)) {
    if (FP_(is_zero)(&R)) C_(xyzz_dbl)(p);
    else C_(xyzz_set_inf)(p);
    return;
  }
  C_(tsqr)(&PP, &P);
  C_(tmul)(&PPP, &P, &PP);
  C_(tmul)(&Q, &U1, &PP);
  FP x3; C_(tsqr)(&x3, &R); FP_(sub)(&x3, &x3, &PPP); FP_(dbl)(&t, &Q); FP_(sub)(&x3, &x3, &t);
  FP_(sub)(&t, &Q, &x3); C_(tmul)(&t, &R, &t);
  FP y3; C_(tmul)(&y3, &S1, &PPP); FP_(sub)(&p->y, &t, &y3);
  p->x = x3;
  C_(tmul)(&t, &p->zz, &q->zz); C_(tmul)(&p->zz, &t, &PP);
  C_(tmul)(&t, &p->zzz, &q->zzz); C_(tmul)(&p->zzz, &t, &PPP);
}

static void C_(xyzz_to_aff)(C_(aff)* r, const C_(xyzz)* p) {
  if (C_(xyzz_is_inf)(p)) { memset(r, 0, sizeof(*r)); r->inf = 1; return; }
  FP izz, izzz;
  FP_(inv)(&izz, &p->zz); FP_(inv)(&izzz, &p->zzz);
  C_(tmul)(&r->x, &p->x, &izz); C_(tmul)(&r->y, &p->y, &izzz); r->inf = 0;
}

/* signed digits of a scalar (4 LE words, value < 2^bits) in windows of c bits:
 * d_w in (-2^(c-1), 2^(c-1)], sum d_w 2^(c w) = k; nw = ceil((bits + 1) / c) windows */
static void C_(recode)(int32_t* d, const uint64_t* k, int c, int nw) {
  int carry = 0;
  for (int w = 0; w < nw; ++w) {
    const int lo = w * c;
    uint32_t v = 0;
    for (int b = 0; b < c; ++b) {
      const int i = lo + b;
      if (i < 256 && ((k[i >> 6] >> (i & 63)) & 1)) v |= 1u << b;
    }
    int32_t x = (int32_t)v + carry;
    if (x > (1 << (c - 1))) { x -= 1 << c; carry = 1; } else { carry = 0; }
    d[w] = x;
  }
}

/* one task: the bucket sum of window w over a point range, for up to three term classes */
typedef struct {
  const C_(aff)* pts;   /* points of the class */
  const int32_t* dig;   /* digits [point][stride] */
  int stride;           /* windows per point in dig */
  size_t lo, hi;        /* point range of this task */
} C_(tclass);

static void C_(bucket_window)(C_(xyzz)* out, C_(xyzz)* bk, int c, int w, const C_(tclass)* cls, int ncls) {
  const size_t nb = (size_t)1 << (c - 1);
  for (size_t b = 0; b < nb; ++b) C_(xyzz_set_inf)(&bk[b]);
  for (int k = 0; k < ncls; ++k) {
    const C_(tclass)* t = &cls[k];
    for (size_t i = t->lo; i < t->hi; ++i) {
      const int32_t d = t->dig[i * (size_t)t->stride + w];
      if (!d || t->pts[i].inf) continue;
      if (d > 0) {
        C_(xyzz_madd)(&bk[d - 1], &t->pts[i].x, &t->pts[i].y);
      } else {
        FP ny; FP_(neg)(&ny, &t->pts[i].y);
        C_(xyzz_madd)(&bk[-d - 1], &t->pts[i].x, &ny);
      }
    }
  }
  /* sum_b (b + 1) bk[b] by running sums from the top */
  C_(xyzz) run, sum;
  C_(xyzz_set_inf)(&run); C_(xyzz_set_inf)(&sum);
  for (size_t b = nb; b-- > 0;) {
    C_(xyzz_add)(&run, &bk[b]);
    C_(xyzz_add)(&sum, &run);
  }
  *out = sum;
}

/* A, B of tuples [offset, offset + n) (seeded counter-mode r_i, as C_(batch_verify)) */
static int C_(batch_verify_tuned)(const uint8_t* cm, const uint8_t* zs, const uint8_t* ys, const uint8_t* pf,
                                  size_t n, const uint8_t* g2b, const uint8_t* tg2b, const uint8_t* seed,
                                  int* ok, uint8_t* a_out, uint8_t* b_out, uint64_t offset, int do_pairing,
                                  int c, size_t chunk) {
  C_(aff2) g2, tg2;
  C_(aff) g1;
  int e;
  if ((e = C_(g2_decode)(&g2, g2b))) return e;
  if ((e = C_(g2_decode)(&tg2, tg2b))) return e;
  C_(generator)(&g1);
  if (c == 0) {  /* auto: about n / 8 buckets per window (16 at n = 2^20, 5 at n = 256) */
    int lg = 0;
    while (((size_t)2 << lg) <= n) ++lg;
    c = lg - 3 < 5 ? 5 : lg - 3 > 16 ? 16 : lg - 3;
  }
  if (c < 4 || c > 20) return KZGO_ERR_ARG;
  if (chunk == 0) chunk = (size_t)1 << 19;
  if (n == 0) {
    *ok = 1;
    C_(aff) inf; memset(&inf, 0, sizeof(inf)); inf.inf = 1;
    if (a_out) C_(g1_encode)(a_out, &inf);
    if (b_out) C_(g1_encode)(b_out, &inf);
    return 0;
  }
  const int wh = (128 + c - 1) / c;  /* windows of a 127-bit r_i, top carry included */
  const int wf = (256 + c - 1) / c;  /* windows of a full Fr scalar (< 2^255) */
  C_(aff)* cpts = (C_(aff)*)malloc(n * sizeof(C_(aff)));
  C_(aff)* ppts = (C_(aff)*)malloc(n * sizeof(C_(aff)));
  int32_t* dr = (int32_t*)malloc(n * (size_t)wh * sizeof(int32_t));
  int32_t* ds = (int32_t*)malloc(n * (size_t)wf * sizeof(int32_t));
  int err = 0;
  FR tsum; FR_(zero)(&tsum);
  #pragma omp parallel num_threads(kzgo_threads())
  {
    FR tloc; FR_(zero)(&tloc);
    #pragma omp for schedule(static)
    for (size_t i = 0; i < n; ++i) {
      int le = C_(g1_decode)(&cpts[i], cm + i * 2 * FPB);
      if (!le) le = C_(g1_decode)(&ppts[i], pf + i * 2 * FPB);
      uint64_t z[4], y[4], ri[4], si[4];
      if (!le) le = C_(fr_decode_raw)(z, zs + 32 * i);
      if (!le) le = C_(fr_decode_raw)(y, ys + 32 * i);
      if (le) {
        #pragma omp critical
        { if (!err) err = le; }
        continue;
      }
      FR rm, zm, ym, s;
      kzgo_randomizer(seed, offset + (uint64_t)i, ri);
      FR_(to_mont)(&rm, ri);
      FR_(to_mont)(&zm, z); FR_(to_mont)(&ym, y);
      FR_(mul)(&s, &rm, &zm); FR_(from_mont)(si, &s);
      FR_(mul)(&s, &rm, &ym); FR_(add)(&tloc, &tloc, &s);
      C_(recode)(dr + i * (size_t)wh, ri, c, wh);
      C_(recode)(ds + i * (size_t)wf, si, c, wf);
    }
    #pragma omp critical
    FR_(add)(&tsum, &tsum, &tloc);
  }
  if (err) { free(cpts); free(ppts); free(dr); free(ds); return err; }
  FR ntm; FR_(neg)(&ntm, &tsum);
  uint64_t traw[4]; FR_(from_mont)(traw, &ntm);
  int32_t dt[64];
  C_(recode)(dt, traw, c, wf);
  /* tasks: (MSM, window, point chunk); MSM#0 windows 0..wh-1 over pi with r; MSM#1 windows
   * 0..wf-1 over C with r (w < wh), pi with s, and (first chunk only) G1 with -t */
  const size_t nch = (n + chunk - 1) / chunk;
  const int ntask = (int)((size_t)(wh + wf) * nch);
  C_(xyzz)* res = (C_(xyzz)*)malloc((size_t)ntask * sizeof(C_(xyzz)));
  C_(aff) gpt[1] = {g1};
  #pragma omp parallel num_threads(kzgo_threads())
  {
    C_(xyzz)* bk = (C_(xyzz)*)malloc(((size_t)1 << (c - 1)) * sizeof(C_(xyzz)));
    #pragma omp for schedule(dynamic, 1)
    for (int t = 0; t < ntask; ++t) {
      const int wi = t / (int)nch;
      const size_t ch = (size_t)(t % (int)nch);
      const size_t lo = ch * chunk, hi = lo + chunk < n ? lo + chunk : n;
      C_(tclass) cls[3];
      int ncls = 0;
      int w;
      if (wi < wh) {  /* MSM#0 */
        w = wi;
        cls[ncls++] = (C_(tclass)){ppts, dr, wh, lo, hi};
      } else {        /* MSM#1 */
        w = wi - wh;
        if (w < wh) cls[ncls++] = (C_(tclass)){cpts, dr, wh, lo, hi};
        cls[ncls++] = (C_(tclass)){ppts, ds, wf, lo, hi};
        if (ch == 0) cls[ncls++] = (C_(tclass)){gpt, dt, wf, 0, 1};
      }
      C_(bucket_window)(&res[t], bk, c, w, cls, ncls);
    }
    free(bk);
  }
  /* Horner over the windows of each MSM (chunk partials summed first) */
  C_(xyzz) acc[2];
  for (int m = 0; m < 2; ++m) {
    const int nw = m == 0 ? wh : wf, base = m == 0 ? 0 : wh;
    C_(xyzz_set_inf)(&acc[m]);
    for (int w = nw - 1; w >= 0; --w) {
      for (int k = 0; k < c; ++k) C_(xyzz_dbl)(&acc[m]);
      for (size_t ch = 0; ch < nch; ++ch) C_(xyzz_add)(&acc[m], &res[(size_t)(base + w) * nch + ch]);
    }
  }
  free(res); free(cpts); free(ppts); free(dr); free(ds);
  C_(aff) A, B;
  C_(xyzz_to_aff)(&A, &acc[0]);
  C_(xyzz_to_aff)(&B, &acc[1]);
  if (a_out) C_(g1_encode)(a_out, &A);
  if (b_out) C_(g1_encode)(b_out, &B);
  *ok = -1;
  if (do_pairing) C_(pairing_check_fast)(&A, &B, &g2, &tg2, ok);
  return 0;
}

/* ================================================================== fast pairing check */
/* Frobenius f -> f^p on the tower (w^2 = v, v^3 = xi): coefficient of w^k conjugated and
 * multiplied by g_k = xi^(k (p - 1) / 6) (computed once) */
typedef struct { T_(fp2) g[6]; int ready; } C_(frobk);
static C_(frobk) C_(frob_consts);

static void C_(frob_init)(void) {
  if (C_(frob_consts).ready) return;
  enum { N = (int)(sizeof(FP) / 8) };
  uint64_t e[N];
  memcpy(e, PRAW, sizeof(e));
  e[0] -= 1;  /* p - 1 (p odd: no borrow) */
  unsigned __int128 rem = 0;
  for (int i = N - 1; i >= 0; --i) {
    const unsigned __int128 cur = (rem << 64) | e[i];
    e[i] = (uint64_t)(cur / 6);
    rem = cur % 6;
  }
  T_(fp2) xi, base;
  T_(fp2_small)(&xi, XI_A, 1);
  T_(fp2_pow)(&base, &xi, e, 64 * N);
  C_(frobk) k;
  T_(fp2_one)(&k.g[0]);
  for (int i = 1; i < 6; ++i) T_(fp2_mul)(&k.g[i], &k.g[i - 1], &base);
  k.ready = 1;
  #pragma omp critical(kzgo_frob)
  C_(frob_consts) = k;
}

static void C_(frob12)(T_(fp12)* r, const T_(fp12)* a) {
  const T_(fp2)* g = C_(frob_consts).g;
  T_(fp2)* dst[6] = {&r->c0.c0, &r->c1.c0, &r->c0.c1, &r->c1.c1, &r->c0.c2, &r->c1.c2};  /* w^0 .. w^5 */
  const T_(fp2)* src[6] = {&a->c0.c0, &a->c1.c0, &a->c0.c1, &a->c1.c1, &a->c0.c2, &a->c1.c2};
  T_(fp12) t;
  T_(fp2)* tdst[6] = {&t.c0.c0, &t.c1.c0, &t.c0.c1, &t.c1.c1, &t.c0.c2, &t.c1.c2};
  for (int k = 0; k < 6; ++k) {
    T_(fp2) c;
    T_(fp2_conj)(&c, src[k]);
    T_(fp2_mul)(tdst[k], &c, &g[k]);
  }
  for (int k = 0; k < 6; ++k) *dst[k] = *tdst[k];
}

static void C_(fp6_sub)(T_(fp6)* r, const T_(fp6)* a, const T_(fp6)* b) {
  T_(fp2_sub)(&r->c0, &a->c0, &b->c0); T_(fp2_sub)(&r->c1, &a->c1, &b->c1); T_(fp2_sub)(&r->c2, &a->c2, &b->c2);
}

/* (a0 + a1 v + a2 v^2)^-1 = (A + B v + C v^2) / F: A = a0^2 - xi a1 a2, B = xi a2^2 - a0 a1,
 * C = a1^2 - a0 a2, F = a0 A + xi (a2 B + a1 C) */
static void C_(fp6_inv)(T_(fp6)* r, const T_(fp6)* a) {
  T_(fp2) A, B, C, F, t, u;
  T_(fp2_mul)(&A, &a->c0, &a->c0); T_(fp2_mul)(&t, &a->c1, &a->c2); T_(fp2_mul_xi)(&t, &t); T_(fp2_sub)(&A, &A, &t);
  T_(fp2_mul)(&B, &a->c2, &a->c2); T_(fp2_mul_xi)(&B, &B); T_(fp2_mul)(&t, &a->c0, &a->c1); T_(fp2_sub)(&B, &B, &t);
  T_(fp2_mul)(&C, &a->c1, &a->c1); T_(fp2_mul)(&t, &a->c0, &a->c2); T_(fp2_sub)(&C, &C, &t);
  T_(fp2_mul)(&t, &a->c2, &B); T_(fp2_mul)(&u, &a->c1, &C); T_(fp2_add)(&t, &t, &u); T_(fp2_mul_xi)(&t, &t);
  T_(fp2_mul)(&F, &a->c0, &A); T_(fp2_add)(&F, &F, &t);
  T_(fp2_inv)(&F, &F);
  T_(fp2_mul)(&r->c0, &A, &F); T_(fp2_mul)(&r->c1, &B, &F); T_(fp2_mul)(&r->c2, &C, &F);
}

/* (c0 + c1 w)^-1 = (c0 - c1 w) / (c0^2 - v c1^2) */
static void C_(fp12_inv)(T_(fp12)* r, const T_(fp12)* a) {
  T_(fp6) t0, t1, ti;
  T_(fp6_mul)(&t0, &a->c0, &a->c0);
  T_(fp6_mul)(&t1, &a->c1, &a->c1);
  T_(fp6_mul_v)(&t1, &t1);
  C_(fp6_sub)(&t0, &t0, &t1);
  C_(fp6_inv)(&ti, &t0);
  T_(fp6_mul)(&r->c0, &a->c0, &ti);
  T_(fp6_mul)(&t1, &a->c1, &ti);
  T_(fp6_neg)(&r->c1, &t1);
}

/* Granger-Scott squaring in the cyclotomic subgroup (the formula of
 * kzg-batch-verification-scheme_amd/tools/gen_bilinear.py cyclo_sqr, in this tower) */
static void C_(fp4_sqr)(T_(fp2)* r0, T_(fp2)* r1, const T_(fp2)* a, const T_(fp2)* b) {
  T_(fp2) t0, t1, s;
  T_(fp2_mul)(&t0, a, a);
  T_(fp2_mul)(&t1, b, b);
  T_(fp2_add)(&s, a, b); T_(fp2_mul)(&s, &s, &s); T_(fp2_sub)(&s, &s, &t0); T_(fp2_sub)(r1, &s, &t1);
  T_(fp2_mul_xi)(&t1, &t1); T_(fp2_add)(r0, &t1, &t0);
}
static void C_(cyc_sqr)(T_(fp12)* r, const T_(fp12)* f) {
  const T_(fp2) z0 = f->c0.c0, z1 = f->c1.c1, z2 = f->c1.c0, z3 = f->c0.c2, z4 = f->c0.c1, z5 = f->c1.c2;
  T_(fp2) t0, t1, t2, t3, t4, t5, u;
  C_(fp4_sqr)(&t0, &t1, &z0, &z1);
  C_(fp4_sqr)(&t2, &t3, &z2, &z3);
  C_(fp4_sqr)(&t4, &t5, &z4, &z5);
  /* r00 = 3 t0 - 2 z0; r11 = 3 t1 + 2 z1; r10 = 3 xi t5 + 2 z2; r02 = 3 t4 - 2 z3; r01 = 3 t2 - 2 z4; r12 = 3 t3 + 2 z5 */
#define KZGO_CYC(dst, tv, zv, sign)                                            \
  do {                                                                         \
    if (sign) T_(fp2_add)(&u, &tv, &zv); else T_(fp2_sub)(&u, &tv, &zv);        \
    T_(fp2_add)(&u, &u, &u); T_(fp2_add)(&dst, &u, &tv);                         \
  } while (0)
  T_(fp12) o;
  KZGO_CYC(o.c0.c0, t0, z0, 0);
  KZGO_CYC(o.c1.c1, t1, z1, 1);
  T_(fp2) xt5; T_(fp2_mul_xi)(&xt5, &t5);
  KZGO_CYC(o.c1.c0, xt5, z2, 1);
  KZGO_CYC(o.c0.c2, t4, z3, 0);
  KZGO_CYC(o.c0.c1, t2, z4, 0);
  KZGO_CYC(o.c1.c2, t3, z5, 1);
#undef KZGO_CYC
  *r = o;
}

/* f^((p^12 - 1) / r * k): easy part, then the hard part as prod_i frob^i(g)^(l_i) by a joint
 * square-and-multiply over a 16-entry table (fexp_gen.h: k = 3 on BLS12-381, as the oracle) */
static void C_(final_exp_fast)(T_(fp12)* r, const T_(fp12)* f) {
  C_(frob_init)();
  T_(fp12) a, b, g;
  C_(fp12_inv)(&a, f);
  T_(fp12_conj)(&b, f);
  T_(fp12_mul)(&a, &b, &a);          /* f^(p^6 - 1) */
  C_(frob12)(&b, &a);
  C_(frob12)(&b, &b);
  T_(fp12_mul)(&g, &b, &a);          /* ^(p^2 + 1) */
  T_(fp12) base[4], tab[16];
  base[0] = g;
  for (int i = 1; i < 4; ++i) C_(frob12)(&base[i], &base[i - 1]);
  for (int i = 0; i < 4; ++i)
    if (HARD_NEG[i]) T_(fp12_conj)(&base[i], &base[i]);  /* cyclotomic inverse */
  T_(fp12_one)(&tab[0]);
  for (int m = 1; m < 16; ++m) {
    int lo = 0;
    while (!((m >> lo) & 1)) ++lo;
    T_(fp12_mul)(&tab[m], &tab[m & (m - 1)], &base[lo]);
  }
  T_(fp12) acc;
  T_(fp12_one)(&acc);
  for (int bit = HARD_BITS - 1; bit >= 0; --bit) {
    C_(cyc_sqr)(&acc, &acc);
    int m = 0;
    for (int i = 0; i < 4; ++i) m |= (int)((HARD_L[i][bit >> 6] >> (bit & 63)) & 1) << i;
    if (m) T_(fp12_mul)(&acc, &acc, &tab[m]);
  }
  *r = acc;
}

/* Miller loop of C_(miller) as a program precomputed from Q alone: every T step's line
 * (slope lam, c = yT - lam xT) or vertical (xT), the squarings and the final conjugation */
enum { C_(OP_SQR) = 0, C_(OP_LINE) = 1, C_(OP_VERT) = 2, C_(OP_CONJ) = 3 };
typedef struct { int op; T_(fp2) lam, c; } C_(mop);
#define KZGO_MAXOPS 320
typedef struct { int n; C_(mop) ops[KZGO_MAXOPS]; } C_(mprog);

static void C_(pre_step)(C_(mprog)* pr, C_(aff2)* T, const C_(aff2)* Q) {
  if (T->inf) { *T = *Q; return; }
  if (Q->inf) return;
  T_(fp2) lam, t, u;
  if (T_(fp2_eq)(&T->x, &Q->x)) {
    T_(fp2_add)(&t, &T->y, &Q->y);
    if (T_(fp2_is_zero)(&t)) {
      C_(mop)* o = &pr->ops[pr->n++];
      o->op = C_(OP_VERT); o->c = T->x;
      memset(T, 0, sizeof(*T)); T->inf = 1; return;
    }
    T_(fp2_mul)(&t, &T->x, &T->x); T_(fp2_add)(&u, &t, &t); T_(fp2_add)(&t, &u, &t);
    T_(fp2_add)(&u, &T->y, &T->y); T_(fp2_inv)(&u, &u); T_(fp2_mul)(&lam, &t, &u);
  } else {
    T_(fp2_sub)(&t, &Q->y, &T->y); T_(fp2_sub)(&u, &Q->x, &T->x);
    T_(fp2_inv)(&u, &u); T_(fp2_mul)(&lam, &t, &u);
  }
  C_(mop)* o = &pr->ops[pr->n++];
  o->op = C_(OP_LINE); o->lam = lam;
  T_(fp2_mul)(&o->c, &lam, &T->x); T_(fp2_sub)(&o->c, &T->y, &o->c);   /* yT - lam xT */
  T_(fp2) x3, y3;
  T_(fp2_mul)(&x3, &lam, &lam); T_(fp2_sub)(&x3, &x3, &T->x); T_(fp2_sub)(&x3, &x3, &Q->x);
  T_(fp2_sub)(&t, &T->x, &x3); T_(fp2_mul)(&y3, &lam, &t); T_(fp2_sub)(&y3, &y3, &T->y);
  T->x = x3; T->y = y3;
}

static void C_(miller_pre)(C_(mprog)* pr, const C_(aff2)* Q) {
  pr->n = 0;
  if (Q->inf) return;
  C_(aff2) T = *Q;
  for (int i = LOOP_BITS - 2; i >= 0; --i) {
    pr->ops[pr->n++].op = C_(OP_SQR);
    C_(aff2) Tc = T;
    C_(pre_step)(pr, &T, &Tc);
    if ((LOOP_WORDS[i / 64] >> (i % 64)) & 1) C_(pre_step)(pr, &T, Q);
  }
#if IS_BLS
  pr->ops[pr->n++].op = C_(OP_CONJ);
#else
  C_(aff2) Q1, Q2;
  C_(frob_twist)(&Q1, Q);
  C_(frob_twist)(&Q2, &Q1);
  T_(fp2_neg)(&Q2.y, &Q2.y);
  C_(pre_step)(pr, &T, &Q1);
  C_(pre_step)(pr, &T, &Q2);
#endif
}

static void C_(miller_eval)(T_(fp12)* f, const C_(mprog)* pr, const C_(aff)* P) {
  T_(fp12_one)(f);
  if (P->inf || pr->n == 0) return;
  for (int k = 0; k < pr->n; ++k) {
    const C_(mop)* o = &pr->ops[k];
    T_(fp12) l;
    if (o->op == C_(OP_SQR)) {
      T_(fp12_mul)(f, f, f);
    } else if (o->op == C_(OP_CONJ)) {
      T_(fp12_conj)(f, f);
    } else if (o->op == C_(OP_LINE)) {
      memset(&l, 0, sizeof(l));
      T_(fp2) b, c;
      T_(fp2_mul_fp)(&b, &o->lam, &P->x);                  /* lam xP */
      T_(fp2_zero)(&c); FP_(neg)(&c.c0, &P->y);            /* -yP */
#if IS_BLS
      l.c0.c0 = o->c; l.c0.c1 = b; l.c1.c1 = c;
#else
      l.c0.c0 = c; l.c1.c0 = b; l.c1.c1 = o->c;
#endif
      T_(fp12_mul)(f, f, &l);
    } else {
      C_(aff2) Tv;
      memset(&Tv, 0, sizeof(Tv));
      Tv.x = o->c;
      C_(vertical)(&l, &Tv, P);
      T_(fp12_mul)(f, f, &l);
    }
  }
}

/* line programs of the last SRS G2 pair seen (the SRS is fixed across a run's batches) */
typedef struct { int valid; uint8_t key[8 * FPB]; C_(mprog) g2, tg2; } C_(pcache_t);
static C_(pcache_t) C_(pcache);

static void C_(pairing_check_fast)(const C_(aff)* A, const C_(aff)* B, const C_(aff2)* g2, const C_(aff2)* tg2,
                                   int* ok) {
  uint8_t key[8 * FPB];
  C_(g2_encode)(key, g2);
  C_(g2_encode)(key + 4 * FPB, tg2);
  const C_(mprog)* pg2;
  const C_(mprog)* ptg2;
  C_(mprog)* own = NULL;
  int hit = 0;
  #pragma omp critical(kzgo_pcache)
  {
    if (!C_(pcache).valid || memcmp(C_(pcache).key, key, sizeof(key))) {
      C_(miller_pre)(&C_(pcache).g2, g2);
      C_(miller_pre)(&C_(pcache).tg2, tg2);
      memcpy(C_(pcache).key, key, sizeof(key));
      C_(pcache).valid = 1;
    }
    own = (C_(mprog)*)malloc(2 * sizeof(C_(mprog)));  /* private copy: the cache may be refilled */
    memcpy(&own[0], &C_(pcache).g2, sizeof(C_(mprog)));
    memcpy(&own[1], &C_(pcache).tg2, sizeof(C_(mprog)));
    hit = 1;
  }
  (void)hit;
  pg2 = &own[0];
  ptg2 = &own[1];
  C_(aff) nB;
  C_(aff_neg)(&nB, B);
  T_(fp12) f1, f2, f;
  C_(miller_eval)(&f1, ptg2, A);
  C_(miller_eval)(&f2, pg2, &nB);
  T_(fp12_mul)(&f, &f1, &f2);
  C_(final_exp_fast)(&f, &f);
  *ok = T_(fp12_is_one)(&f);
  free(own);
}

/* e(P, Q) through the fast Miller program + final exponentiation (tests compare it with the
 * oracle's C_(miller) + plain-pow exponentiation) */
static void C_(pairing_fast)(T_(fp12)* r, const C_(aff)* P, const C_(aff2)* Q) {
  C_(mprog)* pr = (C_(mprog)*)malloc(sizeof(C_(mprog)));
  C_(miller_pre)(pr, Q);
  T_(fp12) f;
  C_(miller_eval)(&f, pr, P);
  free(pr);
  C_(final_exp_fast)(r, &f);
}
