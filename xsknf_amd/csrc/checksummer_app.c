// checksummer_app.c -- the checksummer NF on the MI355X batch path.
//
// Same command line and output as the reference app
// (examples/checksummer/checksummer_user.c:113-260 with
// examples/common/statistics.c): `checksummer [XSKNF_OPTIONS] -- [APP_OPTIONS]`,
// -c REDIRECT|DROP, -i iterations, -q, -x, -a; per-second socket stats;
// cumulative rx written to ./stats.txt on SIGUSR1.  The per-frame callback
// (checksummer_user.c:30-112) is replaced by the GPU batch hook of
// libxsknf_gpu: every rx batch is checksummed by one gfx950 launch.
//
// Extra app options: -g, --gpu-path=ZEROCOPY|STAGED|RESIDENT (include/xsknf_gpu.h);
// -G, --emu-gen=COUNT[:LEN]: with emulated queues (interfaces "emu<k>", whose
// kernel side lives in this process) a generator thread plays the reference
// harness's traffic generator (tests/gen-traffic.lua): COUNT UDP frames of LEN
// bytes (default 64) in its shape per queue, and it drains the tx rings.
// MODE_XDP / MODE_COMBINED need the NF's eBPF object and are not supported.
#define _GNU_SOURCE

#include <errno.h>
#include <getopt.h>
#include <libgen.h>
#include <locale.h>
#include <pthread.h>
#include <stdint.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "../../include/xsknf.h"
#include "../../include/xsknf_gpu.h"

#define NSTATS 13   // counters in struct xsknf_socket_stats

static int opt_action = XSKNF_CSUM_ACTION_REDIRECT;
static int opt_csum_iterations = 1;
static int opt_quiet, opt_extra_stats, opt_app_stats;
static int opt_gpu_path = -1;   // -1: by batch size (RESIDENT up to 128 frames, else ZEROCOPY)
static int opt_gpu_sync;
static int opt_gpu_depth;   // 0: by batch size
static unsigned long opt_gen_count;
static unsigned opt_gen_len = 64;
static volatile sig_atomic_t benchmark_done, stats_requested;
static struct xsknf_config config;

static const struct option long_options[] = {
	{"action", required_argument, 0, 'c'},
	{"csum-iterations", required_argument, 0, 'i'},
	{"quiet", no_argument, 0, 'q'},
	{"extra-stats", no_argument, 0, 'x'},
	{"app-stats", no_argument, 0, 'a'},
	{"gpu-path", required_argument, 0, 'g'},
	{"gpu-sync", no_argument, 0, 's'},
	{"gpu-depth", required_argument, 0, 'd'},
	{"emu-gen", required_argument, 0, 'G'},
	{0, 0, 0, 0},
};

static const struct {
	const char *flags, *text;
} app_help[] = {
	{"-c, --action=REDIRECT|DROP", "send each checksummed frame on (default) or drop it"},
	{"-i, --csum-iterations=N", "sum the UDP payload N times (default 1)"},
	{"-q, --quiet", "no per-second statistics"},
	{"-x, --extra-stats", "also the ring counters"},
	{"-a, --app-stats", "also the syscall counters"},
	{"-g, --gpu-path=PATH", "ZEROCOPY, STAGED or RESIDENT (default RESIDENT up to 128-frame batches, else ZEROCOPY)"},
	{"-s, --gpu-sync", "one batch at a time (default: receive while the GPU works)"},
	{"-d, --gpu-depth=N", "batches in flight per worker, 1-8 (default 4 RESIDENT, else 2 up to 128 frames, else 1)"},
	{"-G, --emu-gen=COUNT[:LEN]", "emulated queues: COUNT generated frames of LEN bytes (default 64) per queue"},
};

static void __attribute__((noreturn)) usage(const char *prog)
{
	fprintf(stderr, "usage: %s [xsknf library options] -- [checksummer options]\nchecksummer options:\n", prog);
	for (size_t k = 0; k < sizeof(app_help) / sizeof(app_help[0]); k++)
		fprintf(stderr, "  %-28s %s\n", app_help[k].flags, app_help[k].text);
	exit(EXIT_FAILURE);
}

static void parse_command_line(int argc, char **argv, char *app_path)
{
	int option_index, c;
	while ((c = getopt_long(argc, argv, "qxasd:i:c:g:G:", long_options, &option_index)) != -1) {
		switch (c) {
		case 'c':
			if (!strcmp(optarg, "REDIRECT")) {
				opt_action = XSKNF_CSUM_ACTION_REDIRECT;
			} else if (!strcmp(optarg, "DROP")) {
				opt_action = XSKNF_CSUM_ACTION_DROP;
			} else {
				fprintf(stderr, "checksummer: action '%s' is neither REDIRECT nor DROP\n", optarg);
				usage(basename(app_path));
			}
			break;
		case 'i':
			opt_csum_iterations = atoi(optarg);
			break;
		case 'q':
			opt_quiet = 1;
			break;
		case 'x':
			opt_extra_stats = 1;
			break;
		case 'a':
			opt_app_stats = 1;
			break;
		case 's':
			opt_gpu_sync = 1;
			break;
		case 'd':
			opt_gpu_depth = atoi(optarg);
			if (opt_gpu_depth < 1 || opt_gpu_depth > XSKNF_MAX_HOOK_DEPTH) {
				fprintf(stderr, "checksummer: GPU depth '%s' is not in 1-%d\n", optarg, XSKNF_MAX_HOOK_DEPTH);
				usage(basename(app_path));
			}
			break;
		case 'g':
			if (!strcmp(optarg, "ZEROCOPY")) {
				opt_gpu_path = XSKNF_GPU_PATH_ZEROCOPY;
			} else if (!strcmp(optarg, "STAGED")) {
				opt_gpu_path = XSKNF_GPU_PATH_STAGED;
			} else if (!strcmp(optarg, "RESIDENT")) {
				opt_gpu_path = XSKNF_GPU_PATH_RESIDENT;
			} else {
				fprintf(stderr, "checksummer: no GPU path named '%s'\n", optarg);
				usage(basename(app_path));
			}
			break;
		case 'G': {
			char *end = NULL;
			opt_gen_count = strtoul(optarg, &end, 10);
			if (end && *end == ':')
				opt_gen_len = (unsigned)strtoul(end + 1, NULL, 10);
			if (opt_gen_len < 42 || opt_gen_len > 3840) {
				fprintf(stderr, "checksummer: generator frame length %u is not in 42-3840\n", opt_gen_len);
				usage(basename(app_path));
			}
			break;
		}
		default:
			usage(basename(app_path));
		}
	}
}

/* ---- generator for emulated queues (the harness's tests/gen-traffic.lua) ---- */

static unsigned long gen_delivered, gen_transmitted;

// Eth 0a:00:00:00:00:01 -> 0a:00:00:00:00:00, IPv4 10.0.0.x -> 172.0.0.1 (ihl 5,
// proto 17), UDP 5000 -> 80, random payload (gen-traffic.lua:16,92-100; the
// checksum is left for the NF, which overwrites it).
static void gen_frame(uint8_t *f, unsigned len, uint64_t *rng)
{
	static const uint8_t hdr[42] = {
		0x0a, 0, 0, 0, 0, 0, 0x0a, 0, 0, 0, 0, 1, 0x08, 0x00,
		0x45, 0, 0, 0, 0, 0, 0, 0, 64, 17, 0, 0, 10, 0, 0, 0, 172, 0, 0, 1,
		0x13, 0x88, 0x00, 0x50, 0, 0, 0, 0,
	};
	for (unsigned i = 42; i < len; i++) {
		*rng ^= *rng << 13;
		*rng ^= *rng >> 7;
		*rng ^= *rng << 17;
		f[i] = (uint8_t)*rng;
	}
	memcpy(f, hdr, 42);
	f[16] = (uint8_t)((len - 14) >> 8);
	f[17] = (uint8_t)(len - 14);
	f[29] = (uint8_t)*rng;          // one of 256 flows
	f[38] = (uint8_t)((len - 34) >> 8);
	f[39] = (uint8_t)(len - 34);
}

static void *gen_loop(void *arg)
{
	(void)arg;
	enum { BURST = 256, TXSTRIDE = 4096 };
	const unsigned queues = config.workers * config.num_interfaces;
	uint8_t *buf = malloc((size_t)BURST * opt_gen_len);
	uint32_t *lens = malloc(sizeof(uint32_t) * BURST);
	uint8_t *txbuf = malloc((size_t)BURST * TXSTRIDE);
	uint32_t *txlens = malloc(sizeof(uint32_t) * BURST);
	unsigned long *left = calloc(queues, sizeof(unsigned long));
	if (!buf || !lens || !txbuf || !txlens || !left)
		goto out;
	for (unsigned q = 0; q < queues; q++)
		left[q] = opt_gen_count;
	uint64_t rng = 0x58534B4EULL;
	unsigned long pending = opt_gen_count * queues;
	while (!benchmark_done) {
		int idle = 1;
		for (unsigned q = 0; q < queues; q++) {
			const unsigned w = q / config.num_interfaces, j = q % config.num_interfaces;
			if (left[q]) {
				const uint32_t n = left[q] < BURST ? (uint32_t)left[q] : BURST;
				for (uint32_t i = 0; i < n; i++) {
					gen_frame(buf + (size_t)i * opt_gen_len, opt_gen_len, &rng);
					lens[i] = opt_gen_len;
				}
				const int got = xsknf_emu_deliver(w, j, buf, lens, n, opt_gen_len);
				if (got < 0)
					goto out;
				left[q] -= (unsigned)got;
				pending -= (unsigned)got;
				__atomic_add_fetch(&gen_delivered, (unsigned long)got, __ATOMIC_RELAXED);
				idle &= got == 0;
			}
			const int sent = xsknf_emu_transmit(w, j, txbuf, txlens, BURST, TXSTRIDE);
			if (sent > 0) {
				__atomic_add_fetch(&gen_transmitted, (unsigned long)sent, __ATOMIC_RELAXED);
				idle = 0;
			}
		}
		if (idle)
			usleep(pending ? 50 : 1000);
	}
out:
	free(buf);
	free(lens);
	free(txbuf);
	free(txlens);
	free(left);
	return NULL;
}

/* ---- statistics (examples/common/statistics.c:33-260) ---- */

static struct xsknf_socket_stats old_stats[XSKNF_MAX_WORKERS][XSKNF_MAX_INTERFACES];
static unsigned long prev_time;

static unsigned long get_nsecs(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec * 1000000000UL + ts.tv_nsec;
}

static void print_socket_stats(const unsigned long *cur, const double *ps, unsigned long dt)
{
	static const char *const names[NSTATS] = {
		"rx", "tx", "rx dropped", "rx invalid", "tx invalid", "rx queue full",
		"fill ring empty", "tx ring empty", "rx empty polls", "fill fail polls",
		"tx wakeup sendtos", "tx trigger sendtos", "opt polls",
	};
	const char *fmt = "%-18s %'-14.0f %'-14lu\n";
	printf("%-14s %-14s %-14.2f\n", "pps", "pkts", dt / 1000000000.);
	for (int i = 0; i < 2; i++)
		printf(fmt, names[i], ps[i], cur[i]);
	if (opt_extra_stats)
		for (int i = 2; i < 8; i++)
			printf(fmt, names[i], ps[i], cur[i]);
	if (opt_app_stats) {
		printf("%-18s %-14s %-14s\n", "", "calls/s", "count");
		for (int i = 8; i < NSTATS; i++)
			printf(fmt, names[i], ps[i], cur[i]);
	}
}

static void dump_stats(void)
{
	const unsigned long now = get_nsecs();
	const unsigned long dt = now - prev_time;
	unsigned long total[NSTATS] = {0};
	double total_ps[NSTATS] = {0};
	prev_time = now;
	for (unsigned w = 0; w < config.workers; w++) {
		for (unsigned j = 0; j < config.num_interfaces; j++) {
			struct xsknf_socket_stats s;
			if (xsknf_get_socket_stats(w, j, &s))
				continue;
			const unsigned long *cur = (const unsigned long *)&s;
			const unsigned long *old = (const unsigned long *)&old_stats[w][j];
			double ps[NSTATS];
			for (int i = 0; i < NSTATS; i++) {
				ps[i] = (cur[i] - old[i]) * 1000000000. / dt;
				total[i] += cur[i];
				total_ps[i] += ps[i];
			}
			char buf[256];
			snprintf(buf, sizeof(buf), " %s@wrk%u", config.interfaces[j], w);
			printf("\n%-19s", buf);
			print_socket_stats(cur, ps, dt);
			old_stats[w][j] = s;
		}
	}
	printf("\n%-19s", " TOTAL");
	print_socket_stats(total, total_ps, dt);
	fflush(stdout);
}

// SIGUSR1: cumulative rx packets to ./stats.txt (statistics.c:219-264)
static void write_stats_file(void)
{
	unsigned long total_rx = 0;
	for (unsigned w = 0; w < config.workers; w++)
		for (unsigned j = 0; j < config.num_interfaces; j++) {
			struct xsknf_socket_stats s;
			if (!xsknf_get_socket_stats(w, j, &s))
				total_rx += s.rx_npkts;
		}
	FILE *f = fopen("./stats.txt", "w");
	if (!f) {
		perror("stats.txt");
		return;
	}
	fprintf(f, "%lu\n", total_rx);
	fclose(f);
}

static void int_exit(int sig)
{
	(void)sig;
	benchmark_done = 1;
}

static void int_usr(int sig)
{
	(void)sig;
	stats_requested = 1;
}

int main(int argc, char **argv)
{
	signal(SIGINT, int_exit);
	signal(SIGTERM, int_exit);
	signal(SIGABRT, int_exit);
	signal(SIGUSR1, int_usr);

	xsknf_parse_args(argc, argv, &config);
	int rc = xsknf_init(&config, NULL);
	if (rc) {
		fprintf(stderr, "ERROR: xsknf_init: %s\n", strerror(-rc));
		return EXIT_FAILURE;
	}
	parse_command_line(argc, argv, argv[0]);
	setlocale(LC_ALL, "");

	const struct xsknf_csum_opts opts = {
		.csum_iterations = opt_csum_iterations,
		.action = opt_action,
		.num_interfaces = config.num_interfaces,
	};
	struct xsknf_gpu_hook *hook = NULL;
	// small rx batches (the reference's default is 64, src/xsknf.c:49): the
	// resident kernel's ring, four batches out.  Set from the NF-level sweep
	// with the feeder pinned apart (tools/hook_default.sh, medians of 5,
	// profiles/r04/nf/): at 64 and 128 frames RESIDENT 21.0 / 21.4 Mpps against
	// 7.9 / 17.5 launched (64 B) and 10.3 / 10.3 against 6.6 / 10.2 (1500 B);
	// from 256 frames the launched hook is level or ahead (64 B 23.5 vs 21.1,
	// 1500 B 11.5 vs 11.0 at 256; 22.5 vs 20.8 and 11.6 vs 10.8 at 1024) -- DESIGN 5.3
	const int small = config.batch_size <= 128;
	if (opt_gpu_path < 0)
		opt_gpu_path = small ? XSKNF_GPU_PATH_RESIDENT : XSKNF_GPU_PATH_ZEROCOPY;
	rc = xsknf_gpu_hook_create(&hook, &opts, config.workers, opt_gpu_path, config.batch_size,
			(uint32_t)config.xsk_frame_size);
	if (rc) {
		fprintf(stderr, "ERROR: GPU hook: %s (%s)\n", strerror(-rc), xsknf_gpu_last_error());
		xsknf_cleanup();
		return EXIT_FAILURE;
	}
	if (opt_gpu_sync)
		xsknf_set_batch_processor((xsknf_batch_processor_fn)xsknf_gpu_hook_process, hook);
	else
		xsknf_set_batch_processor_async((xsknf_batch_submit_fn)xsknf_gpu_hook_submit,
				(xsknf_batch_complete_fn)xsknf_gpu_hook_complete, hook);
	// two in flight pay at the reference's small batches, not from 256 frames on
	// (tools/hook_bench.c: 1500 B x 64 5.8 -> 8.2 Mpps, x 256 13.2 -> 11.8)
	xsknf_set_batch_depth(opt_gpu_depth ? (unsigned)opt_gpu_depth
	                                    : opt_gpu_path == XSKNF_GPU_PATH_RESIDENT ? 4u : (small ? 2u : 1u));
	rc = xsknf_start_workers();
	if (rc) {
		fprintf(stderr, "ERROR: xsknf_start_workers: %s\n", strerror(-rc));
		xsknf_gpu_hook_destroy(hook);
		xsknf_cleanup();
		return EXIT_FAILURE;
	}
	prev_time = get_nsecs();
	pthread_t gen;
	int gen_started = 0;
	if (opt_gen_count)
		gen_started = pthread_create(&gen, NULL, gen_loop, NULL) == 0;

	int err = 0;
	while (!benchmark_done && !err) {
		sleep(1);
		if (stats_requested) {
			stats_requested = 0;
			write_stats_file();
		}
		if (!opt_quiet)
			dump_stats();
		for (unsigned w = 0; w < config.workers && !err; w++)
			err = xsknf_worker_error(w);
	}
	if (err)
		fprintf(stderr, "ERROR: worker stopped: %s (%s)\n", strerror(-err), xsknf_gpu_last_error());
	benchmark_done = 1;
	if (gen_started) {
		pthread_join(gen, NULL);
		fprintf(stderr, "generator: %lu frames delivered, %lu transmitted\n", gen_delivered,
			gen_transmitted);
	}
	xsknf_stop_workers();
	xsknf_gpu_hook_destroy(hook);
	xsknf_cleanup();
	return err ? EXIT_FAILURE : EXIT_SUCCESS;
}
