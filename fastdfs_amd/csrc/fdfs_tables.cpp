// Table construction for the CRC kernels; see fdfs_tables.hpp.
#include "fdfs_tables.hpp"

#include <cstring>
#include <utility>

namespace fdfs {

static inline uint32_t shr8(uint32_t c, int sar)
{
    uint32_t r = c >> 8;
    if (sar && (c & 0x80000000u))
        r |= 0xFF000000u;
    return r;
}

uint32_t crc_step(const CrcTables &t, uint32_t c, uint8_t b)
{
    return t.T[(c ^ b) & 0xFFu] ^ shr8(c, t.sar);
}

static uint32_t adv_bytes(const CrcTables &t, uint32_t v, uint64_t n)
{
    for (uint64_t i = 0; i < n; i++)
        v = crc_step(t, v, 0);
    return v;
}

static uint32_t matvec(const uint32_t cols[32], uint32_t v)
{
    uint32_t r = 0;
    for (int i = 0; i < 32; i++)
        if (v & (1u << i))
            r ^= cols[i];
    return r;
}

uint32_t crc_advance(const CrcTables &t, uint32_t v, uint64_t nbytes)
{
    for (int k = 0; k < 48 && nbytes; k++, nbytes >>= 1)
        if (nbytes & 1)
            v = matvec(t.MPOW[k], v);
    return v;
}

static void byte_tables_of(const CrcTables &t, uint32_t out[4][256], uint64_t n)
{
    // A linear map L splits into 4 byte tables: L(v) = sum_j L(byte_j(v) << 8j).
    // Build from the 32 basis images, then expand (cheap and exact).
    uint32_t img[32];
    for (int i = 0; i < 32; i++)
        img[i] = adv_bytes(t, 1u << i, n);
    for (int j = 0; j < 4; j++)
        for (uint32_t x = 0; x < 256; x++) {
            uint32_t r = 0;
            for (int b = 0; b < 8; b++)
                if (x & (1u << b))
                    r ^= img[8 * j + b];
            out[j][x] = r;
        }
}

bool build_crc_tables(CrcTables &t, bool arithmetic_shift)
{
    std::memset(&t, 0, sizeof(t));
    t.sar = arithmetic_shift ? 1 : 0;
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++)
            c = (c & 1u) ? (0xEDB88320u ^ (c >> 1)) : (c >> 1);
        t.T[i] = c;
    }
    // D[p][x]: 16-byte chunk from state 0, byte p = x, others 0.
    for (int p = 0; p < 16; p++)
        for (uint32_t x = 0; x < 256; x++)
            t.D[p][x] = adv_bytes(t, crc_step(t, 0, (uint8_t)x), (uint64_t)(15 - p));

    // Sign fix: M^16(e_i) must equal D[i/8][bit] for i < 31; the residue at
    // i = 31 is K16 (0 for a logical shift).
    for (int i = 0; i < 32; i++) {
        uint32_t e = 1u << i;
        uint32_t r = adv_bytes(t, e, 16) ^ t.D[i / 8][(e >> (8 * (i / 8))) & 0xFFu];
        if (i < 31 && r != 0)
            return false;
        if (i == 31)
            t.K16 = r;
    }
    if (!t.sar && t.K16 != 0)
        return false;
    // The same for 8-byte chunks: slice-by-8 uses D[8..15].
    for (int i = 0; i < 32; i++) {
        uint32_t e = 1u << i;
        uint32_t r = adv_bytes(t, e, 8) ^ t.D[8 + i / 8][(e >> (8 * (i / 8))) & 0xFFu];
        if (i < 31 && r != 0)
            return false;
        if (i == 31)
            t.K8 = r;
    }
    if (!t.sar && t.K8 != 0)
        return false;

    byte_tables_of(t, t.ADV4032, 4032);
    for (int l = 0; l < 6; l++)
        byte_tables_of(t, t.ADVRED[l], (uint64_t)64 << l);
    byte_tables_of(t, t.ADVSEG, kSegBytes);

    for (int i = 0; i < 32; i++)
        t.MPOW[0][i] = crc_step(t, 1u << i, 0);
    for (int k = 1; k < 48; k++)
        for (int i = 0; i < 32; i++)
            t.MPOW[k][i] = matvec(t.MPOW[k - 1], matvec(t.MPOW[k - 1], 1u << i));

    // The sparse fold's relation S(A) = 0 on every basis vector.
    for (int i = 0; i < 32; i++) {
        uint32_t v = 0;
        for (int k = 0; k < kFoldTerms; k++)
            v ^= crc_advance(t, 1u << i, 16ull * (uint64_t)fold_exp(t.sar != 0, k));
        if (v != 0)
            return false;
    }
    // The lane fold's relation R(A4) = 0 on every basis vector, and Y4: a
    // state c enters a lane's fold as the data dword c ^ (c < 0 ? Y4 : 0),
    // since M^4(c) = crc0(c as 4 data bytes) ^ (c < 0 ? crc0(Y4) : 0).
    for (int i = 0; i < 32; i++) {
        uint32_t v = 0;
        for (int k = 0; k < lane_fold_terms(t.sar != 0); k++)
            v ^= crc_advance(t, 1u << i, 4ull * (uint64_t)lane_fold_exp(t.sar != 0, k));
        if (v != 0)
            return false;
    }
    {
        auto crc0_4 = [&](uint32_t y) {
            return t.D[12][y & 0xFFu] ^ t.D[13][(y >> 8) & 0xFFu] ^ t.D[14][(y >> 16) & 0xFFu] ^ t.D[15][y >> 24];
        };
        const uint32_t k4 = adv_bytes(t, 0x80000000u, 4) ^ crc0_4(0x80000000u);
        // solve crc0_4(y) = k4 over GF(2): eliminate on the basis images
        uint32_t img[32], pre[32];
        for (int i = 0; i < 32; i++) {
            img[i] = crc0_4(1u << i);
            pre[i] = 1u << i;
        }
        uint32_t rhs = k4, y = 0;
        for (int bit = 31, row = 0; bit >= 0; bit--) {
            int piv = -1;
            for (int i = row; i < 32; i++)
                if (img[i] >> bit & 1u) {
                    piv = i;
                    break;
                }
            if (piv < 0)
                return false;  // crc0 of 4 bytes is a bijection
            std::swap(img[row], img[piv]);
            std::swap(pre[row], pre[piv]);
            for (int i = 0; i < 32; i++)
                if (i != row && (img[i] >> bit & 1u)) {
                    img[i] ^= img[row];
                    pre[i] ^= pre[row];
                }
            if (rhs >> bit & 1u) {
                rhs ^= img[row];
                y ^= pre[row];
            }
            row++;
        }
        if (rhs != 0 || crc0_4(y) != k4)
            return false;
        t.Y4 = y;
        if (!t.sar && t.Y4 != 0)
            return false;
    }
    // Self-check the power matrices against direct stepping.
    for (uint64_t n : {(uint64_t)1, (uint64_t)7, (uint64_t)64, (uint64_t)4032, (uint64_t)65539, kSegBytes})
        for (uint32_t v : {0x80000000u, 0x12345678u, 0xFFFFFFFFu})
            if (crc_advance(t, v, n) != adv_bytes(t, v, n))
                return false;
    return true;
}

static uint32_t pow_u32(uint32_t m, uint64_t e)
{
    uint32_t r = 1;
    for (; e; e >>= 1, m *= m)
        if (e & 1)
            r *= m;
    return r;
}

static uint32_t inv_u32(uint32_t m)  // m odd: Newton's iteration for m^-1 mod 2^32
{
    uint32_t x = m;  // correct to 3 bits
    for (int i = 0; i < 5; i++)
        x *= 2 - m * x;
    return x;
}

// Balanced base-256 digits d0..d3 (each in [-128, 127]) with
// sum d_i 256^i == c (mod 2^32).
static void digits4(uint32_t c, int d[4])
{
    int64_t x = c;
    for (int i = 0; i < 4; i++) {
        int v = (int)(x & 0xFF);
        if (v >= 128)
            v -= 256;
        d[i] = v;
        x = (x - v) >> 8;
    }
}

void build_poly_mfma_tables(PolyMfmaTables &t)
{
    std::memset(&t, 0, sizeof(t));
    const uint32_t M[2] = {31u, 33u};
    for (int h = 0; h < 2; h++) {
        int64_t ksum[4] = {0, 0, 0, 0}, ksum64[4] = {0, 0, 0, 0};
        for (int pos = 0; pos < 128; pos++) {
            int d[4];
            digits4(pow_u32(M[h], 127 - pos), d);
            for (int j = 0; j < 4; j++) {
                ksum[j] += d[j];
                if (pos >= 64)
                    ksum64[j] += d[j];
            }
            const int q = pos >> 4, e = pos & 15;
            for (int lane = 0; lane < 64; lane++) {
                const int col = lane & 15, kb = col >> 2, j = col & 3, g = lane >> 4;
                t.B[h][q][lane][e] = (g == kb) ? (int8_t)d[j] : (int8_t)0;
            }
        }
        for (int j = 0; j < 4; j++) {
            t.K[h][j] = (int32_t)(uint32_t)(128 * ksum[j]);
            t.K64[h][j] = (int32_t)(uint32_t)(128 * ksum64[j]);
        }
        // grouped form: 8 steps = 1024 positions per Horner multiply
        int64_t kg[kHornerGroup + 1][4] = {};  // kg[s][j]: digits of plane j over steps >= s
        for (int pos = 1024 - 1; pos >= 0; pos--) {
            int d[4];
            digits4(pow_u32(M[h], 1023 - pos), d);
            const int v = pos >> 4, e = pos & 15;
            for (int j = 0; j < 4; j++) {
                t.BG[h][v][j][e] = (int8_t)d[j];
                kg[pos >> 7][j] += d[j];
            }
        }
        for (int s = kHornerGroup - 2; s >= 0; s--)
            for (int j = 0; j < 4; j++)
                kg[s][j] += kg[s + 1][j];
        for (int j = 0; j < 4; j++) {
            t.KG[h][j] = (int32_t)(uint32_t)(128 * kg[0][j]);
            for (int e = 0; e < kHornerGroup; e++)
                t.KGtail[h][e][j] = (int32_t)(uint32_t)(128 * kg[e][j]);
        }
        t.m1024[h] = pow_u32(M[h], 1024);
        t.m128[h] = pow_u32(M[h], 128);
        t.inv128[h] = inv_u32(t.m128[h]);
        t.m64[h] = pow_u32(M[h], 64);
        t.inv64[h] = inv_u32(t.m64[h]);
    }
}

}  // namespace fdfs
