// Monte-Carlo frame source and error counting on the device.
//   random message bits  : benchmarks/ber_simulation.py:169 (np.random.randint)
//   polar encoder        : src/polar/encoder.py:63-95, src/polar/utils.py:193-229
//   AWGN + BPSK + LLR    : src/channel/awgn.py:27-32, :47, :75, :88, :91-112
//   error counting       : benchmarks/ber_simulation.py:180-189
// Randomness: Philox4x32-10 keyed by (seed, global frame index), so a frame's
// noise does not depend on how frames are sharded over launches or GPUs.
#include "common.hpp"
#include "internal.hpp"

namespace pl {

// one thread per 32 message bits; rows whose 32-bit groups are 16-byte aligned
// (vec) are written as two 16-byte stores of 0/1 bytes instead of 32 byte stores
__global__ void random_bits_kernel(uint64_t seed, int64_t off, int64_t batch, int k, uint8_t* bits, int vec,
                                   int64_t base) {
    const int wpf = (k + 31) / 32;
    const int64_t idx = base + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= batch * wpf) return;
    const int64_t b = idx / wpf;
    const int w = (int)(idx % wpf);
    const uint64_t f = (uint64_t)(off + b);
    const pl_u4 r = philox4x32_10(pl_u4{(uint32_t)w, (uint32_t)f, (uint32_t)(f >> 32), 0xB175B175u},
                                  (uint32_t)seed, (uint32_t)(seed >> 32));
    const uint32_t x = r.x;
    uint8_t* o = bits + b * k + w * 32;
    const int cnt = (k - w * 32) < 32 ? (k - w * 32) : 32;
    if (vec && cnt == 32) {
        uint32_t q[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const uint32_t nib = (x >> (4 * t)) & 0xFu;  // bytes 4t..4t+3 = bits 4t..4t+3
            q[t] = (nib & 1u) | ((nib & 2u) << 7) | ((nib & 4u) << 14) | ((nib & 8u) << 21);
        }
        uint4* o4 = reinterpret_cast<uint4*>(o);
        o4[0] = make_uint4(q[0], q[1], q[2], q[3]);
        o4[1] = make_uint4(q[4], q[5], q[6], q[7]);
        return;
    }
    for (int j = 0; j < cnt; ++j) o[j] = (x >> j) & 1u;
}

// one wavefront per frame, four frames per workgroup (each wavefront its own
// LDS words, no workgroup barrier): u scattered into LDS words from the
// message (4 bytes per lane per load on aligned rows, an LDS OR per set bit at
// its info position), transform in LDS, then 4 codeword bytes per lane per
// store (aligned rows; else bytes).
__global__ void __launch_bounds__(256)
polar_encode_kernel(int N, int K, const int32_t* __restrict__ info_pos, const uint8_t* __restrict__ msg,
                    int64_t batch, uint8_t* __restrict__ cw) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * 4 + wv;
    if (b >= batch) return;
    const int words = N < 32 ? 1 : N / 32;
    uint32_t* X = reinterpret_cast<uint32_t*>(smem) + wv * (words + 2);
    const uint8_t* m = msg + b * K;
    for (int w = lane; w < words; w += 64) X[w] = 0u;
    // LDS runs a wavefront's operations in order: only compiler reordering to stop
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if ((K & 3) == 0 && ((uintptr_t)m & 3) == 0) {
        for (int k0 = 4 * lane; k0 < K; k0 += 256) {
            const uint32_t v = *reinterpret_cast<const uint32_t*>(m + k0);
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                if ((v >> (8 * t)) & 1u) {
                    const int p = info_pos[k0 + t];
                    atomicOr(&X[p >> 5], 1u << (p & 31));
                }
            }
        }
    } else {
        for (int k = lane; k < K; k += 64) {
            if (m[k] & 1) {
                const int p = info_pos[k];
                atomicOr(&X[p >> 5], 1u << (p & 31));
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    for (int w = lane; w < words; w += 64) X[w] = polar_word_transform(X[w]);
    for (int sw = 1; sw < words; sw <<= 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        for (int w = lane; w < words; w += 64)
            if (!(w & sw)) X[w] ^= X[w + sw];
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    uint8_t* o = cw + b * N;
    if ((N & 3) == 0 && ((uintptr_t)o & 3) == 0) {
        uint32_t* o4 = reinterpret_cast<uint32_t*>(o);
        for (int q = lane; q < N / 4; q += 64) {
            const uint32_t x = (X[q >> 3] >> ((q & 7) * 4)) & 15u;  // bits 4q .. 4q+3
            o4[q] = (x & 1u) | ((x & 2u) << 7) | ((x & 4u) << 14) | ((x & 8u) << 21);
        }
    } else {
        for (int j = lane; j < N; j += 64) o[j] = (X[j >> 5] >> (j & 31)) & 1u;
    }
}

// GF(2) block encoder (LDPC valid-codeword encoding, SURVEY §8 f row 3; the
// reference's LDPCEncoder.encode, src/ldpc/encoder.py:56-95, with a generator
// whose rows really span the code): cw[b][j] = parity(msg[b] . G[:, j]).  G is
// bit-packed column-wise as g[w][j] (bit i of word w of column j = G[32w+i][j]),
// so lanes taking consecutive columns read consecutive words.  One wave per
// frame: the message is packed into LDS words by ballots, then each lane XORs
// popcounts over the kw words of its columns.
__global__ void __launch_bounds__(64)
gf2_encode_kernel(const uint32_t* __restrict__ g, int k, int n, const uint8_t* __restrict__ msg, int64_t ldm,
                  int64_t batch, uint8_t* __restrict__ cw, int64_t ldc) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t* mw = reinterpret_cast<uint32_t*>(smem);
    const int64_t b = blockIdx.x;
    if (b >= batch) return;
    const int lane = threadIdx.x;
    const int kw = (k + 31) / 32;
    const uint8_t* m = msg + b * ldm;
    for (int base = 0; base < k; base += 64) {
        const int j = base + lane;
        const unsigned long long bal = __ballot(j < k ? (m[j] & 1) : 0);
        if (lane == 0) {
            mw[base / 32] = (uint32_t)bal;
            if (base / 32 + 1 < kw) mw[base / 32 + 1] = (uint32_t)(bal >> 32);
        }
    }
    __syncthreads();
    uint8_t* o = cw + b * ldc;
    for (int j = lane; j < n; j += 64) {
        uint32_t acc = 0;
        for (int w = 0; w < kw; ++w) acc ^= (uint32_t)__popc(mw[w] & g[(int64_t)w * n + j]);
        o[j] = (uint8_t)(acc & 1u);
    }
}

// two LLRs per thread (one Philox call -> two 53-bit uniforms -> Box-Muller
// pair); with even n and ld and aligned rows (vec) one 2-byte codeword load and
// one 16-byte LLR store per thread
// ROWS: a 2-D grid, blockIdx.x = the frame (b0 + blockIdx.x), blockIdx.y *
// blockDim.x + threadIdx.x = the pair (rows of >= 128 pairs: no 64-bit
// division per thread); otherwise flat over batch * pairs from `base`.
template <bool ROWS>
__global__ void awgn_kernel(const uint8_t* __restrict__ cw, int n, int64_t batch, double sigma,
                            double sigma2, uint64_t seed, int64_t off, double* __restrict__ llr, int64_t ld,
                            int vec, int64_t base) {
    const int ppf = (n + 1) / 2;
    int64_t b;
    int q;
    if constexpr (ROWS) {
        b = base + blockIdx.x;
        q = (int)(blockIdx.y * blockDim.x + threadIdx.x);
        if (q >= ppf) return;
    } else {
        const int64_t idx = base + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if (idx >= batch * ppf) return;
        b = idx / ppf;
        q = (int)(idx % ppf);
    }
    const uint64_t f = (uint64_t)(off + b);
    const pl_u4 r = philox4x32_10(pl_u4{(uint32_t)q, (uint32_t)f, (uint32_t)(f >> 32), 0xA3A3A3A3u},
                                  (uint32_t)seed ^ 0x5bd1e995u, (uint32_t)(seed >> 32));
    const uint64_t a = ((uint64_t)r.y << 32) | r.x, c = ((uint64_t)r.w << 32) | r.z;
    const double u1 = ((double)(a >> 11) + 1.0) * 0x1.0p-53;  // (0, 1]
    const double u2 = (double)(c >> 11) * 0x1.0p-53;           // [0, 1)
    const double rad = sqrt(-2.0 * log(u1));
    double sn, cs;
    sincospi(2.0 * u2, &sn, &cs);
    const double z[2] = {rad * cs, rad * sn};
    double* o = llr + b * ld;
    if (vec) {
        double s0 = 1.0, s1 = 1.0;
        if (cw) {
            const uint16_t pr = *reinterpret_cast<const uint16_t*>(cw + b * n + 2 * q);
            s0 = 1.0 - 2.0 * (double)(pr & 1u);
            s1 = 1.0 - 2.0 * (double)((pr >> 8) & 1u);
        }
        const double y0 = s0 + sigma * z[0], y1 = s1 + sigma * z[1];  // awgn.py:47, :88
        reinterpret_cast<double2*>(o)[q] = make_double2(2.0 * y0 / sigma2, 2.0 * y1 / sigma2);  // awgn.py:75
        return;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int j = 2 * q + h;
        if (j < n) {
            // awgn.py:47 on bit 0 of the codeword byte, as the vector path reads it
            const double s = cw ? 1.0 - 2.0 * (double)(cw[b * n + j] & 1u) : 1.0;
            const double y = s + sigma * z[h];                              // awgn.py:88
            o[j] = 2.0 * y / sigma2;                                        // awgn.py:75
        }
    }
}

PL_DEV void normal_pair(uint64_t seed, uint32_t salt, uint32_t ctr, uint64_t f, double& z0, double& z1) {
    const pl_u4 r = philox4x32_10(pl_u4{ctr, (uint32_t)f, (uint32_t)(f >> 32), salt}, (uint32_t)seed ^ 0x5bd1e995u,
                                  (uint32_t)(seed >> 32));
    const uint64_t a = ((uint64_t)r.y << 32) | r.x, c = ((uint64_t)r.w << 32) | r.z;
    const double u1 = ((double)(a >> 11) + 1.0) * 0x1.0p-53;
    const double u2 = (double)(c >> 11) * 0x1.0p-53;
    const double rad = sqrt(-2.0 * log(u1));
    double sn, cs;
    sincospi(2.0 * u2, &sn, &cs);
    z0 = rad * cs;
    z1 = rad * sn;
}

// Rayleigh block-free fading (src/channel/fading.py:31-63): per bit h = |h_r + i h_i|,
// h_r, h_i ~ N(0, 1/2); y = h s + N(0, sigma); LLR = 2 y h / sigma^2 (CSI at the
// receiver).  One thread per bit, Philox keyed by (seed, global frame, bit).
__global__ void rayleigh_kernel(const uint8_t* __restrict__ cw, int n, int64_t batch, double sigma, double sigma2,
                                uint64_t seed, int64_t off, double* __restrict__ llr, int64_t ld, int64_t base) {
    const int64_t idx = base + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= batch * n) return;
    const int64_t b = idx / n;
    const int j = (int)(idx % n);
    const uint64_t f = (uint64_t)(off + b);
    double hr, hi, z, unused;
    normal_pair(seed, 0xFADE0001u, (uint32_t)j, f, hr, hi);
    normal_pair(seed, 0xFADE0002u, (uint32_t)j, f, z, unused);
    const double h = sqrt(0.5 * (hr * hr + hi * hi));  // |h| with unit-variance components scaled by 1/sqrt(2)
    const double s = cw ? 1.0 - 2.0 * (double)(cw[b * n + j] & 1u) : 1.0;  // bit 0 of the byte, as awgn_kernel
    const double y = h * s + sigma * z;
    llr[b * ld + j] = 2.0 * y * h / sigma2;
}

// Binary symmetric channel (src/channel/bsc.py:33-49): out = bit ^ (u < p),
// u uniform in [0, 1) per bit.
__global__ void bsc_kernel(const uint8_t* __restrict__ cw, int n, int64_t batch, double p, uint64_t seed,
                           int64_t off, uint8_t* __restrict__ out, int64_t ld, int64_t base) {
    const int64_t idx = base + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= batch * n) return;
    const int64_t b = idx / n;
    const int j = (int)(idx % n);
    const uint64_t f = (uint64_t)(off + b);
    const pl_u4 r = philox4x32_10(pl_u4{(uint32_t)j, (uint32_t)f, (uint32_t)(f >> 32), 0xB5CB5C00u},
                                  (uint32_t)seed ^ 0x5bd1e995u, (uint32_t)(seed >> 32));
    const double u = (double)((((uint64_t)r.y << 32) | r.x) >> 11) * 0x1.0p-53;
    const uint8_t bit = cw ? (uint8_t)(cw[b * n + j] & 1u) : (uint8_t)0;
    out[b * ld + j] = bit ^ (uint8_t)(u < p ? 1 : 0);
}

// HIP caps a launch at 2^32 work-items per grid dimension: element-wise
// launches over more work-items (1 M frames x 8192 bits) go in chunks of 2^30.
constexpr int64_t kChunkItems = 1LL << 30;

template <typename Launch>
static hipError_t chunked(int64_t tot, Launch&& launch) {
    for (int64_t base = 0; base < tot; base += kChunkItems) {
        const int64_t items = tot - base < kChunkItems ? tot - base : kChunkItems;
        launch(dim3((unsigned)((items + 255) / 256)), base);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t rayleigh_launch(const uint8_t* cw, int n, int64_t batch, double sigma, double sigma2, uint64_t seed,
                           int64_t off, double* llr, int64_t ld, hipStream_t s) {
    return chunked(batch * n, [&](dim3 grid, int64_t base) {
        hipLaunchKernelGGL(rayleigh_kernel, grid, dim3(256), 0, s, cw, n, batch, sigma, sigma2, seed, off, llr, ld,
                           base);
    });
}

hipError_t bsc_launch(const uint8_t* cw, int n, int64_t batch, double p, uint64_t seed, int64_t off, uint8_t* out,
                      int64_t ld, hipStream_t s) {
    return chunked(batch * n, [&](dim3 grid, int64_t base) {
        hipLaunchKernelGGL(bsc_kernel, grid, dim3(256), 0, s, cw, n, batch, p, seed, off, out, ld, base);
    });
}

// Bit / frame error counts of dec against ref (low bit of each byte), per-block
// partial sums -> 3 integer atomics.  cpr = 16-byte chunks per row when both
// row sets are 16-byte aligned with a width multiple of 16 (else 0: bytes):
//   cpr a power of two <= 64: 64 / cpr rows per wavefront, one chunk per lane;
//   otherwise: one row per wavefront, chunks (cpr > 0) or bytes strided by 64.
__global__ void __launch_bounds__(256)
count_errors_kernel(const uint8_t* __restrict__ ref, int64_t ldr, const uint8_t* __restrict__ dec,
                    int64_t ldd, int width, int64_t batch, int64_t* counts, int cpr) {
    __shared__ unsigned long long part[2][4];
    const int wave = threadIdx.x / 64, lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * 4, w0 = (int64_t)blockIdx.x * 4 + wave;
    auto chunk_err = [&](int64_t b, int c) -> int {
        const uint4 x = reinterpret_cast<const uint4*>(ref + b * ldr)[c];
        const uint4 y = reinterpret_cast<const uint4*>(dec + b * ldd)[c];
        constexpr uint32_t M = 0x01010101u;
        return __popc((x.x ^ y.x) & M) + __popc((x.y ^ y.y) & M) + __popc((x.z ^ y.z) & M) +
               __popc((x.w ^ y.w) & M);
    };
    unsigned long long be = 0, fe = 0;
    if (cpr > 0 && cpr <= 64 && (cpr & (cpr - 1)) == 0) {
        const int rpw = 64 / cpr;
        const int64_t r = lane / cpr;
        // two row groups per trip: their loads are in flight together
        for (int64_t b0 = w0 * rpw; b0 < batch; b0 += 2 * waves * rpw) {
            const int64_t b = b0 + r, b2 = b + waves * rpw;
            int e = b < batch ? chunk_err(b, lane % cpr) : 0;
            int e2 = b2 < batch ? chunk_err(b2, lane % cpr) : 0;
            for (int sh = cpr / 2; sh > 0; sh >>= 1) {
                e += __shfl_xor(e, sh);
                e2 += __shfl_xor(e2, sh);
            }
            if (lane % cpr == 0) {
                be += (unsigned)(e + e2);
                fe += (e > 0 ? 1 : 0) + (e2 > 0 ? 1 : 0);
            }
        }
    } else {
        for (int64_t b = w0; b < batch; b += waves) {
            int e = 0;
            if (cpr > 0) {
                for (int c = lane; c < cpr; c += 64) e += chunk_err(b, c);
            } else {
                for (int j = lane; j < width; j += 64) e += (ref[b * ldr + j] & 1) != (dec[b * ldd + j] & 1);
            }
            for (int sh = 32; sh > 0; sh >>= 1) e += __shfl_xor(e, sh);
            if (lane == 0) {
                be += (unsigned)e;
                fe += e > 0 ? 1 : 0;
            }
        }
    }
    for (int sh = 32; sh > 0; sh >>= 1) {
        be += __shfl_xor(be, sh);
        fe += __shfl_xor(fe, sh);
    }
    if (lane == 0) { part[0][wave] = be; part[1][wave] = fe; }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long sb = 0, sf = 0;
        for (int w = 0; w < 4; ++w) { sb += part[0][w]; sf += part[1][w]; }
        atomicAdd(reinterpret_cast<unsigned long long*>(counts + 0), sb);
        atomicAdd(reinterpret_cast<unsigned long long*>(counts + 1), sf);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0)
        atomicAdd(reinterpret_cast<unsigned long long*>(counts + 2), (unsigned long long)batch);
}

hipError_t random_bits_launch(uint64_t seed, int64_t off, int64_t batch, int k, uint8_t* bits,
                              hipStream_t s) {
    const int vec = (k % 16 == 0) && (((uintptr_t)bits & 15) == 0);
    return chunked(batch * ((k + 31) / 32), [&](dim3 grid, int64_t base) {
        hipLaunchKernelGGL(random_bits_kernel, grid, dim3(256), 0, s, seed, off, batch, k, bits, vec, base);
    });
}

hipError_t polar_encode_launch(int N, int K, const int32_t* info_pos, const uint8_t* msg, int64_t batch,
                               uint8_t* cw, hipStream_t s) {
    if (batch == 0) return hipSuccess;
    const int words = N < 32 ? 1 : N / 32;
    hipLaunchKernelGGL(polar_encode_kernel, dim3((unsigned)((batch + 3) / 4)), dim3(256), 4 * (words + 2) * 4, s, N,
                       K, info_pos, msg, batch, cw);
    return hipGetLastError();
}

hipError_t gf2_encode_launch(const uint32_t* g, int k, int n, const uint8_t* msg, int64_t ldm, int64_t batch,
                             uint8_t* cw, int64_t ldc, hipStream_t s) {
    if (batch == 0) return hipSuccess;
    const int kw = (k + 31) / 32;
    hipLaunchKernelGGL(gf2_encode_kernel, dim3((unsigned)batch), dim3(64), (size_t)kw * 4 + 8, s, g, k, n, msg, ldm,
                       batch, cw, ldc);
    return hipGetLastError();
}

hipError_t awgn_launch(const uint8_t* cw, int n, int64_t batch, double sigma, double sigma2, uint64_t seed,
                       int64_t off, double* llr, int64_t ld, hipStream_t s) {
    const int vec = (n % 2 == 0) && (ld % 2 == 0) && (((uintptr_t)llr & 15) == 0) && (((uintptr_t)cw & 1) == 0);
    const int ppf = (n + 1) / 2;
    if (ppf >= 128) {
        const int t = ppf >= 256 ? 256 : 128;
        const unsigned gy = (unsigned)((ppf + t - 1) / t);
        const int64_t fmax = (int64_t)1 << 24;  // frames per launch (grid x)
        for (int64_t b0 = 0; b0 < batch; b0 += fmax) {
            const int64_t nf = batch - b0 < fmax ? batch - b0 : fmax;
            hipLaunchKernelGGL(awgn_kernel<true>, dim3((unsigned)nf, gy), dim3(t), 0, s, cw, n, batch, sigma, sigma2,
                               seed, off, llr, ld, vec, b0);
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    return chunked(batch * ppf, [&](dim3 grid, int64_t base) {
        hipLaunchKernelGGL(awgn_kernel<false>, grid, dim3(256), 0, s, cw, n, batch, sigma, sigma2, seed, off, llr, ld,
                           vec, base);
    });
}

// CRC append (src/polar/utils.py:86-125 crc_encode, bit-serial MSB first, zero
// initial register): msg[b][k_data + t] = bit (crc_len-1-t) of the CRC register
// of msg[b][0:k_data].  One thread per frame (k_data sequential steps).
__global__ void __launch_bounds__(256)
crc_append_kernel(uint8_t* __restrict__ msg, int64_t ld, int64_t batch, int k_data, int crc_len, uint32_t poly) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    uint8_t* m = msg + b * ld;
    const uint32_t top = 1u << (crc_len - 1), mask = crc_len == 32 ? 0xFFFFFFFFu : ((1u << crc_len) - 1u);
    uint32_t crc = 0;
    for (int i = 0; i < k_data; ++i) {
        crc ^= (uint32_t)(m[i] & 1u) << (crc_len - 1);
        crc = (crc & top) ? ((crc << 1) ^ poly) : (crc << 1);
        crc &= mask;
    }
    for (int t = 0; t < crc_len; ++t) m[k_data + t] = (uint8_t)((crc >> (crc_len - 1 - t)) & 1u);
}

hipError_t crc_append_launch(uint8_t* msg, int64_t ld, int64_t batch, int k_data, int crc_len, uint32_t poly,
                             hipStream_t s) {
    if (batch == 0) return hipSuccess;
    hipLaunchKernelGGL(crc_append_kernel, dim3((unsigned)((batch + 255) / 256)), dim3(256), 0, s, msg, ld, batch,
                       k_data, crc_len, poly);
    return hipGetLastError();
}

hipError_t count_errors_launch(const uint8_t* ref, int64_t ldr, const uint8_t* dec, int64_t ldd, int width,
                               int64_t batch, int64_t* counts, hipStream_t s) {
    if (batch == 0) return hipSuccess;
    const bool vec = width % 16 == 0 && ldr % 16 == 0 && ldd % 16 == 0 && ((uintptr_t)ref & 15) == 0 &&
                     ((uintptr_t)dec & 15) == 0;
    const int cpr = vec ? width / 16 : 0;
    const int rpw = (cpr > 0 && cpr <= 64 && (cpr & (cpr - 1)) == 0) ? 64 / cpr : 1;  // rows per wavefront
    int64_t blocks = (batch + 8 * rpw - 1) / (8 * rpw);
    if (blocks > 512) blocks = 512;  // two same-address atomics per block: keep them few
    hipLaunchKernelGGL(count_errors_kernel, dim3((unsigned)blocks), dim3(256), 0, s, ref, ldr, dec, ldd, width,
                       batch, counts, cpr);
    return hipGetLastError();
}

}  // namespace pl
