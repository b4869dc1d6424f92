/*
 * multi_config4.c -- BASELINE config 4 through the C host's multi-device calls,
 * from C (include/xsknf_gpu.h xsknf_gpu_multi_*), as a C host that owns a global
 * batch on one device would drive them.  Measurement / test infrastructure: it
 * links the CPU oracle (oracle/build/libcsum_oracle.so, pinned to the
 * reference's own function by tests/test_ref_pin.py) as the checker.
 *
 *   multi_config4 [frames (default 8388608)] [devices (default: all)]
 *
 * The batch: IMIX 64 / 570 / 1500 B frames (7:4:1, shuffled), one per 2 KiB
 * chunk at +256 (aligned mode), Eth / IPv4 / UDP headers, random payload, built
 * on the host and copied to device 0.  Then, over devices 0..D-1:
 *   1. span path: xsknf_gpu_multi_scatter (each shard's UMEM span and rebased
 *      descriptors, grouped ncclSend / ncclRecv from device 0), _process (one
 *      launch per device, in place on the shards), _counters (ncclAllReduce);
 *   2. frames only, out and back: xsknf_gpu_multi_scatter_packed, then
 *      xsknf_gpu_multi_return into device 0's UMEM and a verdict array.
 * Checked against the oracle's pass over a host copy of the batch: the
 * all-reduced counters (frames, bytes, drops, forwards, the written checks
 * summed and weighted by global offset) and, after the return, device 0's UMEM
 * and verdicts, every byte.  Prints one JSON line; exit status 0 iff all match.
 */
#define _GNU_SOURCE
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "xsknf_gpu.h"

struct oracle_desc { uint64_t addr; uint32_t len; uint32_t options; };
struct oracle_opts { int32_t csum_iterations; int32_t action; uint32_t num_interfaces; uint32_t reserved; };
void oracle_process_batch(uint8_t *umem, const struct oracle_desc *descs, uint32_t n, uint32_t ingress,
			  const struct oracle_opts *o, int32_t *verdicts, uint32_t batch);

#define CHUNK 2048u
#define HEADROOM 256u

static uint64_t rng_state = 0x58534B4E;   /* the SURVEY's seed, as a xorshift64* state */
static uint64_t rnd(void)
{
	rng_state ^= rng_state >> 12;
	rng_state ^= rng_state << 25;
	rng_state ^= rng_state >> 27;
	return rng_state * 0x2545F4914F6CDD1DULL;
}

static double now(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

#define HIP_OK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
	fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(2); } } while (0)
#define XS_OK(x) do { int r_ = (x); if (r_) { \
	fprintf(stderr, "%s: %d (%s)\n", #x, r_, xsknf_gpu_last_error()); exit(2); } } while (0)

static void put16(uint8_t *p, uint16_t v) { p[0] = v >> 8; p[1] = v & 0xff; }   /* network order */

/* One frame of `len` bytes at p: Ethernet / IPv4 (ihl 5) / UDP 5000 -> 80,
 * UDP check 0 (the checksummer writes it), random payload. */
static void make_frame(uint8_t *p, uint32_t len, uint32_t flow)
{
	for (uint32_t i = 0; i < len; i += 8) {
		uint64_t r = rnd();
		memcpy(p + i, &r, len - i < 8 ? len - i : 8);
	}
	static const uint8_t mac[12] = {0x02, 0, 0, 0, 0, 2, 0x02, 0, 0, 0, 0, 1};
	memcpy(p, mac, 12);
	put16(p + 12, 0x0800);
	uint8_t *ip = p + 14;
	ip[0] = 0x45; ip[1] = 0;
	put16(ip + 2, (uint16_t)(len - 14));
	put16(ip + 4, 0); put16(ip + 6, 0);
	ip[8] = 64; ip[9] = 17;
	put16(ip + 10, 0);
	ip[12] = 10; ip[13] = 0; ip[14] = 0; ip[15] = (uint8_t)flow;
	ip[16] = 172; ip[17] = 0; ip[18] = 0; ip[19] = 1;
	uint8_t *udp = ip + 20;
	put16(udp, 5000); put16(udp + 2, 80);
	put16(udp + 4, (uint16_t)(len - 34));
	put16(udp + 6, 0);
}

/* The counters xsknf_gpu_multi_counters reports, over a whole host batch after
 * its pass (xsknf_amd/multi.py expected_counters). */
static void host_counters(const uint8_t *umem, uint64_t umem_size, const struct xsknf_gpu_desc *d,
			  const int32_t *v, uint64_t n, uint64_t *out)
{
	memset(out, 0, sizeof(uint64_t) * XSKNF_GPU_MULTI_COUNTERS);
	for (uint64_t i = 0; i < n; i++) {
		const uint64_t off = (d[i].addr & XSKNF_GPU_UNALIGNED_BUF_ADDR_MASK) +
				     (d[i].addr >> XSKNF_GPU_UNALIGNED_BUF_OFFSET_SHIFT);
		out[0] += 1;
		out[1] += d[i].len;
		out[2] += v[i] == -1;
		out[3] += v[i] >= 0;
		if (d[i].len >= 42 && off <= umem_size && d[i].len <= umem_size - off) {
			const uint64_t ck = umem[off + 40] | (uint64_t)umem[off + 41] << 8;
			out[4] += ck;
			out[5] += ck * (off % 65521 + 1);
		}
	}
}

int main(int argc, char **argv)
{
	const uint64_t n = argc > 1 ? strtoull(argv[1], NULL, 0) : 8388608ull;
	int ndev = 0;
	XS_OK(xsknf_gpu_device_count(&ndev));
	if (argc > 2 && atoi(argv[2]) > 0 && atoi(argv[2]) < ndev)
		ndev = atoi(argv[2]);
	const uint64_t umem_size = n * CHUNK;

	/* the batch on the host: IMIX lengths 7:4:1, shuffled (Fisher-Yates) */
	uint8_t *host = malloc(umem_size), *ref = malloc(umem_size), *back = malloc(umem_size);
	struct xsknf_gpu_desc *descs = malloc(sizeof(*descs) * n);
	int32_t *ov = malloc(sizeof(int32_t) * n), *gv = malloc(sizeof(int32_t) * n);
	uint32_t *lens = malloc(sizeof(uint32_t) * n);
	if (!host || !ref || !back || !descs || !ov || !gv || !lens) {
		fprintf(stderr, "out of host memory\n");
		return 2;
	}
	for (uint64_t i = 0; i < n; i++)
		lens[i] = i % 12 < 7 ? 64 : (i % 12 < 11 ? 570 : 1500);
	for (uint64_t i = n; i > 1; i--) {
		const uint64_t j = rnd() % i;
		const uint32_t t = lens[i - 1]; lens[i - 1] = lens[j]; lens[j] = t;
	}
	memset(host, 0, umem_size);
	uint64_t frame_bytes = 0;
	for (uint64_t i = 0; i < n; i++) {
		descs[i].addr = i * CHUNK + HEADROOM;
		descs[i].len = lens[i];
		descs[i].options = 0;
		frame_bytes += lens[i];
		make_frame(host + descs[i].addr, lens[i], (uint32_t)(rnd() & 0xff));
	}
	memcpy(ref, host, umem_size);
	const uint32_t mean = (uint32_t)(frame_bytes / (n ? n : 1));

	/* the reference answer: the oracle's pass over the whole batch, -i 1 REDIRECT, 1 interface */
	const struct oracle_opts oo = {1, 0, 1, 0};
	oracle_process_batch(ref, (const struct oracle_desc *)descs, (uint32_t)n, 0, &oo, ov, 64);
	uint64_t want[XSKNF_GPU_MULTI_COUNTERS];
	host_counters(ref, umem_size, descs, ov, n, want);

	/* the global batch on device 0 */
	uint8_t *umem = NULL;
	int32_t *verdicts = NULL;
	HIP_OK(hipSetDevice(0));
	HIP_OK(hipMalloc((void **)&umem, umem_size));
	HIP_OK(hipMalloc((void **)&verdicts, sizeof(int32_t) * (n ? n : 1)));
	HIP_OK(hipMemcpy(umem, host, umem_size, hipMemcpyHostToDevice));

	struct xsknf_gpu_multi *m = NULL;
	XS_OK(xsknf_gpu_multi_create(&m, NULL, ndev));
	const struct xsknf_csum_opts o = {1, XSKNF_CSUM_ACTION_REDIRECT, 1, 0};

	/* 1. the span path, in place on the shards, the counters all-reduced */
	double t_span = 0;
	float *ms = calloc(ndev, sizeof(float));
	XS_OK(xsknf_gpu_multi_scatter(m, 0, umem, umem_size, descs, n, &t_span));
	XS_OK(xsknf_gpu_multi_process(m, 0, &o, 1500, mean, ms));
	uint64_t got[XSKNF_GPU_MULTI_COUNTERS];
	XS_OK(xsknf_gpu_multi_counters(m, got));
	const int counters_match = !memcmp(got, want, sizeof(got));
	float step_max = 0;
	for (int k = 0; k < ndev; k++)
		step_max = ms[k] > step_max ? ms[k] : step_max;

	/* 2. frames only, out and back into device 0's UMEM (still the original batch);
	 * packed_calls_wall_ms: the two calls on the host's clock, with their host-side
	 * planning and descriptor staging (the calls' own `seconds` exclude them).
	 * step_us_max above is this process's first pass (no warm-up). */
	double t_pack = 0, t_ret = 0;
	const double t0 = now();
	XS_OK(xsknf_gpu_multi_scatter_packed(m, 0, umem, umem_size, descs, n, &t_pack));
	XS_OK(xsknf_gpu_multi_return(m, 0, &o, 1500, mean, umem, verdicts, ms, &t_ret));
	const double t_trip = now() - t0;
	uint64_t moved = 0;
	for (int k = 0; k < ndev; k++) {
		struct xsknf_gpu_shard_info si;
		XS_OK(xsknf_gpu_multi_shard_info(m, k, &si));
		moved += si.span_hi - si.span_lo;
	}
	XS_OK(xsknf_gpu_multi_destroy(m));
	HIP_OK(hipSetDevice(0));
	HIP_OK(hipMemcpy(back, umem, umem_size, hipMemcpyDeviceToHost));
	HIP_OK(hipMemcpy(gv, verdicts, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
	const int umem_match = !memcmp(back, ref, umem_size);
	const int verdicts_match = !memcmp(gv, ov, sizeof(int32_t) * n);

	printf("{\"frames\": %llu, \"devices\": %d, \"frame_bytes\": %llu, \"span_scatter_ms\": %.3f, "
	       "\"step_us_max\": %.2f, \"counters_match\": %s, \"packed_scatter_ms\": %.3f, \"packed_bytes\": %llu, "
	       "\"return_ms\": %.3f, \"packed_calls_wall_ms\": %.3f, \"root_umem_match\": %s, \"verdicts_match\": %s}\n",
	       (unsigned long long)n, ndev, (unsigned long long)frame_bytes, t_span * 1e3, step_max * 1e3,
	       counters_match ? "true" : "false", t_pack * 1e3, (unsigned long long)moved, t_ret * 1e3,
	       t_trip * 1e3, umem_match ? "true" : "false", verdicts_match ? "true" : "false");
	HIP_OK(hipFree(umem));
	HIP_OK(hipFree(verdicts));
	return counters_match && umem_match && verdicts_match ? 0 : 1;
}
