// moments.cpp — host contraction of pair moments into DenseFactor::linearize's packed
// 13 x 13 information (moments.hpp).  Eight pairs at a time, one per SIMD lane
// (structure of arrays): every coefficient and every sum below is an 8-wide vector op,
// the C matrices' structural zeros are skipped by fixed masks.  Two builds of the same
// code, chosen once per process: AVX-512 (the GPU box's EPYC) and the host's baseline.
// Deterministic on a given host; agrees with the per-row device linearization to
// rounding (~1e-15 relative, tests/test_moments.py).
#include "moments.hpp"

#include <algorithm>
#include <cstdint>
#include <cstring>

namespace fmxh {
namespace {

constexpr int L = 8;
typedef double v8d __attribute__((vector_size(64)));  // GCC vector extension: one zmm (or 2 ymm / 4 xmm)
struct alignas(64) V {
  v8d x;  // lane l: x[l]
};
inline void vset(V& o, double x) { o.x = v8d{x, x, x, x, x, x, x, x}; }
inline void vmul(V& o, const V& a, const V& b) { o.x = a.x * b.x; }
inline void vfma(V& o, const V& a, const V& b) { o.x += a.x * b.x; }
inline void vsub(V& o, const V& a, const V& b) { o.x = a.x - b.x; }
inline void vneg(V& o, const V& a) { o.x = -a.x; }
inline void vadd(V& o, const V& a, const V& b) { o.x = a.x + b.x; }

// epsilon_{abc} as (b, c) pairs with sign for each a: (y x z)_a = y_b z_c - y_c z_b
constexpr int kE1[3] = {1, 2, 0}, kE2[3] = {2, 0, 1};

// The structural nonzeros of C, row by row (13 output rows, feature columns):
//   plane features: 0 r0 | 1-3 n x q0 | 4-6 n | 7-15 n_b p_j,d (7 + 3b + d)
//   point features: 0-2 e0 | 3-5 p_i | 6-8 p_j | 9 one (axis a's residual row: e0_a)
// Only these entries of C are written and read.
struct NzList {
  int8_t n[13];
  int8_t j[13][16];
};
constexpr NzList plane_nz() {
  NzList L{};
  for (int a = 0; a < 3; ++a) {
    const int b = kE1[a], c = kE2[a];
    int m = 0;
    L.j[a][m++] = (int8_t)(1 + a);
    L.j[a][m++] = (int8_t)(4 + b);
    L.j[a][m++] = (int8_t)(4 + c);
    for (int d = 0; d < 3; ++d) {
      L.j[a][m++] = (int8_t)(7 + 3 * b + d);
      L.j[a][m++] = (int8_t)(7 + 3 * c + d);
    }
    L.n[a] = (int8_t)m;
    L.j[3 + a][0] = (int8_t)(4 + a);
    L.n[3 + a] = 1;
    m = 0;
    for (int e = 0; e < 3; ++e) {
      L.j[6 + a][m++] = (int8_t)(7 + 3 * e + b);
      L.j[6 + a][m++] = (int8_t)(7 + 3 * e + c);
    }
    L.n[6 + a] = (int8_t)m;
    for (int e = 0; e < 3; ++e) L.j[9 + a][e] = (int8_t)(4 + e);
    L.n[9 + a] = 3;
  }
  int m = 0;
  L.j[12][m++] = 0;
  for (int k = 4; k < 16; ++k) L.j[12][m++] = (int8_t)k;
  L.n[12] = (int8_t)m;
  return L;
}
constexpr NzList point_nz(int a) {
  NzList L{};
  for (int x = 0; x < 3; ++x) {
    L.j[x][0] = (int8_t)(3 + kE1[x]);
    L.j[x][1] = (int8_t)(3 + kE2[x]);
    L.n[x] = 2;
    L.j[3 + x][0] = 9;
    L.n[3 + x] = 1;
    L.j[6 + x][0] = (int8_t)(6 + kE1[x]);
    L.j[6 + x][1] = (int8_t)(6 + kE2[x]);
    L.n[6 + x] = 2;
    L.j[9 + x][0] = 9;
    L.n[9 + x] = 1;
  }
  int m = 0;
  L.j[12][m++] = (int8_t)a;
  for (int k = 3; k < 10; ++k) L.j[12][m++] = (int8_t)k;
  L.n[12] = (int8_t)m;
  return L;
}
constexpr NzList kPlNz = plane_nz();
constexpr NzList kPtNz[3] = {point_nz(0), point_nz(1), point_nz(2)};

inline int packed16(int r, int c) { return r * 16 - r * (r - 1) / 2 + (c - r); }

// One block of eight pairs, structure of arrays (MomBatch::data).
struct Block {
  V pl[16][16];        // plane moments (symmetric, full)
  V pt[10][10];        // point moments (features 0..9)
  V Ri0[9], ti0[3], Rj0[9], tj0[3], M0[9], v0[3];  // reference poses, M0 = R_i0^T R_j0, v0 = R_i0^T (t_j0 - t_i0)
};
constexpr size_t kBlockD = sizeof(Block) / sizeof(double);

// G += C Phi C^T over the structural nonzeros of C (upper triangle, x <= y).  Row x of
// tmp = C Phi lives in NF vector registers while C's nonzeros of row x stream past;
// then row x of G takes tmp[x] . C[y] over row y's nonzeros.
template <int NF, int LD>
inline __attribute__((always_inline)) void sandwich(const V (&C)[13][16], const V (&Phi)[LD][LD], const NzList& nz,
                                                    V (&G)[13][13]) {
  V tmp[16];
  for (int x = 0; x < 13; ++x) {
    V acc[NF];
#pragma GCC unroll 16
    for (int k = 0; k < NF; ++k) vset(acc[k], 0.0);
    for (int q = 0; q < nz.n[x]; ++q) {
      const int j = nz.j[x][q];
      const V cx = C[x][j];
#pragma GCC unroll 16
      for (int k = 0; k < NF; ++k) vfma(acc[k], cx, Phi[j][k]);
    }
#pragma GCC unroll 16
    for (int k = 0; k < NF; ++k) tmp[k] = acc[k];
    for (int y = x; y < 13; ++y) {
      V a;
      vset(a, 0.0);
      for (int q = 0; q < nz.n[y]; ++q) {
        const int j = nz.j[y][q];
        vfma(a, tmp[j], C[y][j]);
      }
      vadd(G[x][y], G[x][y], a);
    }
  }
}

inline void gather_pose(const Pose* const* T, int nl, V (&R)[9], V (&t)[3]) {
  for (int l = 0; l < L; ++l) {
    const double* m = T[l < nl ? l : 0]->m;
    for (int r = 0; r < 3; ++r) {
      for (int c = 0; c < 3; ++c) R[3 * r + c].x[l] = m[4 * r + c];
      t[r].x[l] = m[4 * r + 3];
    }
  }
}
// M = R_i^T R_j, v = R_i^T (t_j - t_i)
inline __attribute__((always_inline)) void rel(const V (&Ri)[9], const V (&ti)[3], const V (&Rj)[9], const V (&tj)[3],
                                               V (&M)[9], V (&v)[3]) {
  for (int b = 0; b < 3; ++b)
    for (int c = 0; c < 3; ++c) {
      vmul(M[3 * b + c], Ri[b], Rj[c]);
      vfma(M[3 * b + c], Ri[3 + b], Rj[3 + c]);
      vfma(M[3 * b + c], Ri[6 + b], Rj[6 + c]);
    }
  V d[3];
  for (int k = 0; k < 3; ++k) vsub(d[k], tj[k], ti[k]);
  for (int b = 0; b < 3; ++b) {
    vmul(v[b], Ri[b], d[0]);
    vfma(v[b], Ri[3 + b], d[1]);
    vfma(v[b], Ri[6 + b], d[2]);
  }
}

void prepare_block(Block& B, int nl, const double* const* mom, const Pose* const* Ti0, const Pose* const* Tj0) {
  for (int l = 0; l < L; ++l) {
    const double* m = mom[l < nl ? l : 0];
    for (int r = 0; r < 16; ++r)
      for (int c = r; c < 16; ++c) B.pl[r][c].x[l] = B.pl[c][r].x[l] = m[packed16(r, c)];
    for (int r = 0; r < 10; ++r)
      for (int c = r; c < 10; ++c) B.pt[r][c].x[l] = B.pt[c][r].x[l] = m[kMomPacked + packed16(r, c)];
  }
  gather_pose(Ti0, nl, B.Ri0, B.ti0);
  gather_pose(Tj0, nl, B.Rj0, B.tj0);
  rel(B.Ri0, B.ti0, B.Rj0, B.tj0, B.M0, B.v0);
}

inline __attribute__((always_inline)) void eval_block(const Block& B, int nl, const Pose* const* Ti,
                                                      const Pose* const* Tj, double inv, double* G) {
  V Ri[9], ti[3], Rj[9], tj[3];
  gather_pose(Ti, nl, Ri, ti);
  gather_pose(Tj, nl, Rj, tj);
  V Gs[13][13];
  for (int x = 0; x < 13; ++x)
    for (int y = x; y < 13; ++y) vset(Gs[x][y], 0.0);
  V C[13][16];
  // ---- plane rows
  {
    V M[9], v[3], dM[9], dv[3];
    rel(Ri, ti, Rj, tj, M, v);
    for (int k = 0; k < 9; ++k) vsub(dM[k], M[k], B.M0[k]);
    for (int k = 0; k < 3; ++k) vsub(dv[k], v[k], B.v0[k]);
    for (int a = 0; a < 3; ++a) {
      // rows 0-2: (n x q)_a = n_b q_c - n_c q_b, (b, c) = kE1/kE2[a]
      const int b = kE1[a], c = kE2[a];
      vset(C[a][1 + a], 1.0);
      for (int dd = 0; dd < 3; ++dd) {  // n x (dM p_j): n_b dM[c][d] p_d - n_c dM[b][d] p_d
        C[a][7 + 3 * b + dd] = dM[3 * c + dd];
        vneg(C[a][7 + 3 * c + dd], dM[3 * b + dd]);
      }
      C[a][4 + b] = dv[c];  // n x dv
      vneg(C[a][4 + c], dv[b]);
      vset(C[3 + a][4 + a], -1.0);  // -n
      // rows 6-8: (p_j x m)_a = p_b m_c - p_c m_b, m_k = sum_e M[e][k] n_e
      for (int e = 0; e < 3; ++e) {
        C[6 + a][7 + 3 * e + b] = M[3 * e + c];
        vneg(C[6 + a][7 + 3 * e + c], M[3 * e + b]);
        C[9 + a][4 + e] = M[3 * e + a];  // m_a
      }
    }
    vset(C[12][0], -1.0);  // -r = -(r0 + n.(dM p_j) + n.dv)
    for (int b = 0; b < 3; ++b) {
      for (int dd = 0; dd < 3; ++dd) vneg(C[12][7 + 3 * b + dd], dM[3 * b + dd]);
      vneg(C[12][4 + b], dv[b]);
    }
    sandwich<16, 16>(C, B.pl, kPlNz, Gs);
  }
  // ---- point rows, one world axis at a time
  {
    V dRi[9], dRj[9], dt[3];
    for (int k = 0; k < 9; ++k) {
      vsub(dRi[k], Ri[k], B.Ri0[k]);
      vsub(dRj[k], Rj[k], B.Rj0[k]);
    }
    for (int k = 0; k < 3; ++k) {
      V a1, a2;
      vsub(a1, tj[k], B.tj0[k]);
      vsub(a2, ti[k], B.ti0[k]);
      vsub(dt[k], a1, a2);
    }
    for (int a = 0; a < 3; ++a) {
      for (int x = 0; x < 3; ++x) {
        const int b = kE1[x], c = kE2[x];
        // H_i[x] = (p_i x rho)_x, rho = -R_i[a]: p_b rho_c - p_c rho_b
        vneg(C[x][3 + b], Ri[3 * a + c]);
        C[x][3 + c] = Ri[3 * a + b];
        vneg(C[3 + x][9], Ri[3 * a + x]);
        // H_j[x] = (p_j x R_j[a])_x
        C[6 + x][6 + b] = Rj[3 * a + c];
        vneg(C[6 + x][6 + c], Rj[3 * a + b]);
        C[9 + x][9] = Rj[3 * a + x];
      }
      vset(C[12][a], -1.0);  // -r_a
      for (int dd = 0; dd < 3; ++dd) {
        vneg(C[12][6 + dd], dRj[3 * a + dd]);
        C[12][3 + dd] = dRi[3 * a + dd];
      }
      vneg(C[12][9], dt[a]);
      sandwich<10, 10>(C, B.pt, kPtNz[a], Gs);
    }
  }
  // whitening (1 / sigma^2), packed upper 13 x 13 + error
  const double s = inv * inv;
  for (int l = 0; l < nl; ++l) {
    double* g = G + 92 * (size_t)l;
    int o = 0;
    for (int x = 0; x < 13; ++x)
      for (int y = x; y < 13; ++y) g[o++] = Gs[x][y].x[l] * s;
    g[91] = 0.5 * g[90];
  }
}

// MomBatch::data viewed as 64-byte-aligned blocks (the vector was over-allocated by 8)
inline const Block* blocks(const MomBatch& b) {
  const uintptr_t p = reinterpret_cast<uintptr_t>(b.data.data());
  return reinterpret_cast<const Block*>((p + 63) & ~(uintptr_t)63);
}

void eval_generic(const MomBatch& b, const Pose* const* Ti, const Pose* const* Tj, double inv, double* G) {
  const Block* B = blocks(b);
  for (int k = 0; k < b.n; k += L)
    eval_block(B[k / L], std::min(L, b.n - k), Ti + k, Tj + k, inv, G + 92 * (size_t)k);
}
__attribute__((target("avx512f,fma"))) void eval_512(const MomBatch& b, const Pose* const* Ti, const Pose* const* Tj,
                                                     double inv, double* G) {
  const Block* B = blocks(b);
  for (int k = 0; k < b.n; k += L)
    eval_block(B[k / L], std::min(L, b.n - k), Ti + k, Tj + k, inv, G + 92 * (size_t)k);
}
bool has_avx512() {
  static const bool v = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("fma");
  return v;
}

}  // namespace

void mom_prepare(MomBatch& b, int n, const double* const* mom, const Pose* const* Ti0, const Pose* const* Tj0) {
  b.n = std::max(n, 0);
  const int nb = (b.n + L - 1) / L;
  // 64-byte alignment for the vector loads: over-allocate and align the view
  b.data.resize((size_t)nb * kBlockD + 8);
  Block* B = const_cast<Block*>(blocks(b));
  for (int k = 0; k < nb; ++k)
    prepare_block(B[k], std::min(L, b.n - L * k), mom + L * k, Ti0 + L * k, Tj0 + L * k);
}

void mom_eval(const MomBatch& b, const Pose* const* Ti, const Pose* const* Tj, double inv, double* G) {
  if (b.n <= 0) return;
  if (has_avx512()) eval_512(b, Ti, Tj, inv, G);
  else eval_generic(b, Ti, Tj, inv, G);
}

}  // namespace fmxh
