// Host-side construction of every CRC table the kernels use.
//
// All of them are derived from ONE function, the single-byte step of
// CRC32_ex (libfastcommon, called at storage/storage_dio.c:467):
//     c' = crc_table[(c ^ b) & 0xFF] ^ (c >> 8)
// where `>>` is arithmetic for the signed-int state libfastcommon declares
// and logical for an unsigned state.  Flipping `sar` regenerates the slice,
// advance and GF(2) power tables; no kernel code changes.
#pragma once
#include <cstdint>
#ifndef __host__
#define __host__
#define __device__
#endif

namespace fdfs {

// The unit crc_seg_kernel's waves divide the files into (a wave folds its
// consecutive segments of one file as one run), and poly_seg_kernel's per
// wave (64 lanes' spans).
constexpr uint64_t kSegBytes = 128 * 1024;

// The sparse fold of crc_seg_kernel: S(y) = sum_k y^e_k,
// k = 0..4, with S(A) = 0 for A = the advance by 16 zero bytes of each shift
// variant (a 5-term multiple of A's minimal polynomial, found by a
// meet-in-the-middle search over the powers of A, scripts/fold_search.py;
// build_crc_tables re-verifies it on the 32 basis vectors).  Because
// A^e_4 = sum_{k<4} A^e_k, the CRC contribution of a 16-byte vector at
// distance >= e_4 vectors from the end moves to the four vectors
// e_4 - e_k further on, by XOR alone.  The gaps e_4 - e_3 (203 / 145) are
// >= 64: a wave folds 64 consecutive vectors at once.
constexpr int kFoldTerms = 5;
__host__ __device__ constexpr int fold_exp(bool sar, int k)
{
    return sar ? (k == 0 ? 0 : k == 1 ? 332 : k == 2 ? 344 : k == 3 ? 372 : 575)
               : (k == 0 ? 0 : k == 1 ? 89 : k == 2 ? 117 : k == 3 ? 155 : 300);
}

// The lane fold of sig_hash_kernel: R(y) = sum_k y^r_k, the
// minimal polynomial of A4 = the advance by 4 zero bytes (degree 32; 13 terms
// for the arithmetic shift, 15 for the logical one; Gaussian elimination over
// the powers of A4, scripts/fold_search.py lane).  Because A4^32 =
// sum_{k<last} A4^r_k, a lane folds its file's dwords as
// c'_j = x_j ^ sum_{k<last} c'_{j - (32 - r_k)} in 32 registers -- no table
// lookup -- and takes the crc0 of the last 32 c' (after a correction inside
// that window) with the slice-by-16 tables.  build_crc_tables re-verifies
// R(A4) = 0 on the 32 basis vectors.
constexpr int kLaneFoldMaxTerms = 15;
__host__ __device__ constexpr int lane_fold_terms(bool sar) { return sar ? 13 : 15; }
__host__ __device__ constexpr int lane_fold_exp(bool sar, int k)
{
    constexpr int es[13] = {0, 1, 2, 3, 6, 7, 11, 19, 20, 22, 24, 31, 32};
    constexpr int el[15] = {0, 1, 2, 4, 5, 7, 8, 10, 11, 12, 16, 22, 23, 26, 32};
    return sar ? es[k] : el[k];
}

// Zero-input byte step M (advance by one zero byte) is GF(2)-linear in the
// state for both shift semantics, which is what every table below relies on.
struct CrcTables {
    uint32_t T[256];          // byte step table (reflected 0xEDB88320)
    uint32_t D[16][256];      // slice-by-16: byte x at chunk position p -> state at chunk end
    uint32_t K16;             // chain16 sign fix: M^16(c) = sum_j D[j][byte_j(c)] ^ (c<0 ? K16 : 0)
    uint32_t K8;              // chain8 sign fix: M^8(c) = sum_j D[8+j][byte_j(c)] ^ (c<0 ? K8 : 0)
    uint32_t ADV4032[4][256]; // advance by 4032 zero bytes (a 4 KiB block - a lane's 64-byte piece)
    uint32_t ADVRED[6][4][256]; // advance by 64<<t bytes, t = 0..5 (wave reduction tree)
    uint32_t ADVSEG[4][256];  // advance by one segment (kSegBytes; crc_tab_kernel's runs)
    uint32_t MPOW[48][32];    // columns of M^(2^k), k = 0..47 (arbitrary advance)
    uint32_t Y4;              // lane fold: the dword y with crc0(y) = M^4(e_31) ^ crc0(e_31) (0 for a logical shift)
    int sar;                  // 1 = arithmetic shift (signed state)
};

// simple_hash_ex (M = 31) and Time33Hash_ex (M = 33) on the i8 matrix cores
// (see sig_hash_kernel): over one 128-byte step the hash advances as
//   h' = M^128 h + sum_pos M^(127 - pos) b_pos   (mod 2^32),
// a dot product with fixed coefficients.  Each coefficient is split into
// four balanced base-256 digits (int8), one per output "plane"; byte data
// enters the i8 MFMA as b ^ 0x80 = b - 128 and the 128 * sum(digits) term is
// added back per step (K).  B[h][q][lane] is the lane's 16-byte B operand for
// vector q of the step: block-diagonal over the 4 lane groups, so one
// v_mfma_i32_16x16x64_i8 yields the 4 planes of 64 files' 16-byte dots.
struct PolyMfmaTables {
    int8_t B[2][8][64][16];  // [hash 0 = M 31, 1 = M 33][vector q][lane][k element]
    int32_t K[2][4];         // per plane: 128 * sum over the step of the digits
    uint32_t m128[2];        // M^128 mod 2^32
    uint32_t inv128[2];      // M^-128 mod 2^32
    // the same for 64-byte steps (vectors q = 4..7 of B: coefficients M^63..M^0)
    int32_t K64[2][4];
    uint32_t m64[2];
    uint32_t inv64[2];
    // Horner once per group of kHornerGroup 128-byte steps (sig_hash_kernel):
    // BG[h][v][j] = digit plane j of the 16 coefficients M^(1023 - 16 v - e)
    // of vector v of the group (the block-diagonal lane rows, compacted),
    // KG = 128 * sum of a plane's digits over the group, m1024 = M^1024, and
    // KGtail[h][e][j] = the part of KG that belongs to the steps after the
    // first e, taken back when the last group ran only e steps.
    int8_t BG[2][64][4][16];
    int32_t KG[2][4];
    int32_t KGtail[2][8][4];
    uint32_t m1024[2];
};
constexpr int kHornerGroup = 8;  // 128-byte steps per Horner multiply

void build_poly_mfma_tables(PolyMfmaTables &t);

// Returns false if an internal identity check fails (never expected).
bool build_crc_tables(CrcTables &t, bool arithmetic_shift);

// Host reference of the step (used by the table builder and self-checks).
uint32_t crc_step(const CrcTables &t, uint32_t c, uint8_t b);
uint32_t crc_advance(const CrcTables &t, uint32_t v, uint64_t nbytes);

}  // namespace fdfs
