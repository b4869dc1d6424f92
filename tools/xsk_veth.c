// xsk_veth.c -- config 1 harness: the checksummer NF over a veth pair.
//
// Measurement / test infrastructure.  The per-frame NF is the reference's own
// xsknf_packet_processor() compiled from its verbatim lines
// (oracle/_ref/libcsum_ref.so, loaded at run time) where that library was
// built, else the CPU restatement it is pinned to ("nf" in the output says
// which); the two-phase mode uses the restatement's batch hook.  Everything runs inside a private network
// namespace created here (unshare), so nothing outside this process is
// touched: veth pair xg0 <-> xn0, the xsknf runtime (include/xsknf.h) on xn0
// in XDP skb mode (-S, hence copy mode), AF_PACKET generators on xg0.
//
// Modes
//   --search     zero-loss rate search like tests/test-drop-cpu.py:99-122 of
//                the reference (binary search over the offered rate, loss =
//                (sent - rx_npkts) / sent <= 0.1 %, rx_npkts from the runtime's
//                socket stats as the reference reads stats.txt)
//   --check OUT  send every frame of --frames once (REDIRECT), capture what
//                comes back on xg0 and write it to OUT for byte comparison
//
// Frames come from a file written by tools/config1.py (xsknf_amd.frames):
//   "XSKF" u32 count, then per frame u32 len + len bytes.
// Prints one JSON line.
#define _GNU_SOURCE

#include <arpa/inet.h>
#include <dlfcn.h>
#include <errno.h>
#include <linux/if_ether.h>
#include <linux/if_link.h>
#include <linux/if_packet.h>
#include <net/if.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include "../include/xsknf.h"
#include "../xsknf_amd/csrc/rt_netlink.h"

#ifndef PACKET_QDISC_BYPASS
#define PACKET_QDISC_BYPASS 20
#endif
#ifndef PACKET_IGNORE_OUTGOING
#define PACKET_IGNORE_OUTGOING 23
#endif

// the oracle's reference-shaped callback (oracle/csum_oracle.c)
void oracle_nf_set_options(int32_t csum_iterations, int32_t action, uint32_t num_interfaces);
int oracle_nf_packet_processor(void *pkt, unsigned len, unsigned ingress_ifindex);
int oracle_nf_batch_submit(void *user, unsigned worker, void *umem, uint64_t umem_size,
		const struct xdp_desc *descs, uint32_t n, unsigned ingress, int32_t *verdicts, uint64_t *ticket);
int oracle_nf_batch_complete(void *user, unsigned worker, void *umem, uint64_t ticket);

struct frames {
	uint32_t n;
	uint32_t *len;
	uint8_t **data;
};

static struct frames fr;
static volatile int gen_stop;
static volatile double gen_rate;         // offered frames/s, all generators together
static int gen_threads = 3;
static unsigned long gen_sent[64] __attribute__((aligned(64)));
static int gen_ifindex;

static double now_s(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static int load_frames(const char *path)
{
	FILE *f = fopen(path, "rb");
	if (!f)
		return -errno;
	char magic[4];
	if (fread(magic, 1, 4, f) != 4 || memcmp(magic, "XSKF", 4) || fread(&fr.n, 4, 1, f) != 1) {
		fclose(f);
		return -EINVAL;
	}
	fr.len = calloc(fr.n, sizeof(*fr.len));
	fr.data = calloc(fr.n, sizeof(*fr.data));
	if (!fr.len || !fr.data) {
		fclose(f);
		return -ENOMEM;
	}
	for (uint32_t i = 0; i < fr.n; i++) {
		if (fread(&fr.len[i], 4, 1, f) != 1 || fr.len[i] > 9216) {
			fclose(f);
			return -EINVAL;
		}
		fr.data[i] = malloc(fr.len[i] ? fr.len[i] : 1);
		if (!fr.data[i] || fread(fr.data[i], 1, fr.len[i], f) != fr.len[i]) {
			fclose(f);
			return -EINVAL;
		}
	}
	fclose(f);
	return 0;
}

static int pin_self(int cpu)
{
	cpu_set_t s;
	CPU_ZERO(&s);
	CPU_SET(cpu, &s);
	return pthread_setaffinity_np(pthread_self(), sizeof(s), &s);
}

static int packet_socket(int ifindex, int proto)
{
	int fd = socket(AF_PACKET, SOCK_RAW | SOCK_CLOEXEC, htons(proto));
	if (fd < 0)
		return -errno;
	struct sockaddr_ll sll = {.sll_family = AF_PACKET, .sll_protocol = htons(proto),
				  .sll_ifindex = ifindex};
	if (bind(fd, (struct sockaddr *)&sll, sizeof(sll))) {
		close(fd);
		return -errno;
	}
	return fd;
}

struct gen_arg {
	int id;
	int cpu;
};

// paced sendmmsg of the frame set, round robin, 32 frames per call
static void *generator(void *p)
{
	const struct gen_arg *a = p;
	pin_self(a->cpu);
	int fd = packet_socket(gen_ifindex, 0);
	if (fd < 0)
		return NULL;
	int one = 1;
	setsockopt(fd, SOL_PACKET, PACKET_QDISC_BYPASS, &one, sizeof(one));
	enum { B = 32 };
	struct mmsghdr msg[B];
	struct iovec iov[B];
	uint32_t next = (uint32_t)a->id * 7919u;
	double t0 = now_s();
	unsigned long sent = 0;
	while (!gen_stop) {
		const double rate = gen_rate / gen_threads;
		if (rate <= 0) {
			usleep(1000);
			t0 = now_s();
			sent = 0;
			continue;
		}
		// pace: do not run ahead of rate * elapsed
		const double due = (now_s() - t0) * rate;
		if ((double)sent > due) {
			continue;
		}
		for (int i = 0; i < B; i++) {
			const uint32_t k = next++ % fr.n;
			iov[i].iov_base = fr.data[k];
			iov[i].iov_len = fr.len[k];
			memset(&msg[i], 0, sizeof(msg[i]));
			msg[i].msg_hdr.msg_iov = &iov[i];
			msg[i].msg_hdr.msg_iovlen = 1;
		}
		const int r = sendmmsg(fd, msg, B, 0);
		if (r > 0) {
			sent += (unsigned long)r;
			__atomic_fetch_add(&gen_sent[a->id * 8], (unsigned long)r, __ATOMIC_RELAXED);
		}
	}
	close(fd);
	return NULL;
}

static unsigned long total_sent(void)
{
	unsigned long s = 0;
	for (int i = 0; i < gen_threads; i++)
		s += __atomic_load_n(&gen_sent[i * 8], __ATOMIC_RELAXED);
	return s;
}

static unsigned long nf_rx(void)
{
	struct xsknf_socket_stats st;
	if (xsknf_get_socket_stats(0, 0, &st))
		return 0;
	return st.rx_npkts;
}

// one trial at `rate` frames/s for `secs`: returns loss, fills sent / rcvd
static double trial(double rate, double secs, unsigned long *sent_out, unsigned long *rx_out,
		double *achieved)
{
	const unsigned long s0 = total_sent(), r0 = nf_rx();
	const double t0 = now_s();
	gen_rate = rate;
	usleep((useconds_t)(secs * 1e6));
	gen_rate = 0;
	const double t1 = now_s();
	usleep(200000);   // drain what is in flight
	const unsigned long sent = total_sent() - s0, rx = nf_rx() - r0;
	*sent_out = sent;
	*rx_out = rx;
	*achieved = sent / (t1 - t0);
	return sent ? (double)((long)sent - (long)rx) / (double)sent : 1.0;
}

static int capture(const char *out_path, double secs, unsigned long *got)
{
	int fd = packet_socket(gen_ifindex, ETH_P_ALL);
	if (fd < 0)
		return fd;
	int one = 1;
	setsockopt(fd, SOL_PACKET, PACKET_IGNORE_OUTGOING, &one, sizeof(one));
	struct timeval tv = {0, 100000};
	setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
	int bufsz = 64 << 20;
	setsockopt(fd, SOL_SOCKET, SO_RCVBUFFORCE, &bufsz, sizeof(bufsz));
	FILE *f = fopen(out_path, "wb");
	if (!f) {
		close(fd);
		return -errno;
	}
	uint32_t count = 0;
	fwrite("XSKF", 1, 4, f);
	fwrite(&count, 4, 1, f);
	// send everything once (paced low enough not to lose any), then drain
	int tx = packet_socket(gen_ifindex, 0);
	if (tx < 0) {
		fclose(f);
		close(fd);
		return tx;
	}
	static uint8_t buf[10000];
	static const uint8_t our_src[6] = {0x0a, 0, 0, 0, 0, 0x01};   // tools/config1.py frames
	uint32_t sent = 0, ours = 0;
	const double end_by = now_s() + secs;
	double last_rx = now_s();
	while (now_s() < end_by) {
		if (sent < fr.n && send(tx, fr.data[sent], fr.len[sent], 0) >= 0)
			sent++;
		// drain; once everything is sent, wait (100 ms receive timeout) for stragglers
		for (;;) {
			const ssize_t n = recv(fd, buf, sizeof(buf), sent < fr.n ? MSG_DONTWAIT : 0);
			if (n < 0)
				break;
			const uint32_t l = (uint32_t)n;
			fwrite(&l, 4, 1, f);
			fwrite(buf, 1, l, f);
			count++;
			if (l >= 12 && !memcmp(buf + 6, our_src, 6))
				ours++;
			last_rx = now_s();
			if (sent < fr.n)
				break;
		}
		// kernel-originated frames (IPv6 ND on link up) also come back: only ours count
		if (sent >= fr.n && (ours >= fr.n || now_s() - last_rx > 1.0))
			break;
	}
	fseek(f, 4, SEEK_SET);
	fwrite(&count, 4, 1, f);
	fclose(f);
	close(tx);
	close(fd);
	*got = count;
	return 0;
}

int main(int argc, char **argv)
{
	const char *frames_path = NULL, *check_out = NULL;
	int iterations = 1, action_drop = 1, search = 0, nf_cpu = 0, batch = 64, two_phase = 0, use_poll = 0;
	double max_mpps = 4.0, step_mpps = 0.05, trial_s = 2.0;
	for (int i = 1; i < argc; i++) {
		const char *a = argv[i];
		const char *v = i + 1 < argc ? argv[i + 1] : NULL;
		if (!strcmp(a, "--frames") && v) { frames_path = v; i++; }
		else if (!strcmp(a, "--check") && v) { check_out = v; action_drop = 0; i++; }
		else if (!strcmp(a, "--search")) { search = 1; }
		else if (!strcmp(a, "--iterations") && v) { iterations = atoi(v); i++; }
		else if (!strcmp(a, "--redirect")) { action_drop = 0; }
		else if (!strcmp(a, "--max-mpps") && v) { max_mpps = atof(v); i++; }
		else if (!strcmp(a, "--step-mpps") && v) { step_mpps = atof(v); i++; }
		else if (!strcmp(a, "--trial-s") && v) { trial_s = atof(v); i++; }
		else if (!strcmp(a, "--generators") && v) { gen_threads = atoi(v); i++; }
		else if (!strcmp(a, "--batch") && v) { batch = atoi(v); i++; }
		else if (!strcmp(a, "--two-phase")) { two_phase = 1; }
		else if (!strcmp(a, "--poll")) { use_poll = 1; }
		else {
			fprintf(stderr, "usage: %s --frames F [--search|--check OUT] [--iterations k] "
				"[--redirect] [--max-mpps M] [--step-mpps S] [--trial-s T] [--generators G] "
				"[--batch B] [--two-phase] [--poll]\n", argv[0]);
			return 2;
		}
	}
	if (!frames_path || (!search && !check_out) || gen_threads < 1 || gen_threads > 8)
		return 2;
	int rc = load_frames(frames_path);
	if (rc) {
		fprintf(stderr, "frames: %s\n", strerror(-rc));
		return 1;
	}
	if (unshare(CLONE_NEWNET)) {
		printf("{\"error\": \"unshare(CLONE_NEWNET): %s\"}\n", strerror(errno));
		return 3;
	}
	if ((rc = xsknf_nl_create_veth("xg0", "xn0"))) {
		printf("{\"error\": \"veth: %s\"}\n", strerror(-rc));
		return 3;
	}
	gen_ifindex = (int)if_nametoindex("xg0");
	const int nf_ifindex = (int)if_nametoindex("xn0");
	if (xsknf_nl_link_up(gen_ifindex) || xsknf_nl_link_up(nf_ifindex)) {
		printf("{\"error\": \"link up\"}\n");
		return 3;
	}

	// the NF: checksummer_user.c with the reference per-frame callback, -S, 1 worker
	char ifname[] = "xn0";
	struct xsknf_config cfg;
	memset(&cfg, 0, sizeof(cfg));
	cfg.interfaces[0] = ifname;
	cfg.bind_flags[0] = XDP_USE_NEED_WAKEUP;
	cfg.num_interfaces = 1;
	cfg.workers = 1;
	cfg.working_mode = MODE_AF_XDP;
	cfg.xdp_flags = XDP_FLAGS_UPDATE_IF_NOEXIST | XDP_FLAGS_SKB_MODE;
	cfg.batch_size = (uint32_t)batch;
	cfg.xsk_frame_size = 4096;
	cfg.poll = use_poll;
	oracle_nf_set_options(iterations, action_drop, 1);
	const char *nf = "port";
	if (two_phase) {   // the NF as a two-phase batch hook: batches in flight across worker passes
		xsknf_set_batch_processor_async(oracle_nf_batch_submit, oracle_nf_batch_complete, NULL);
	} else {
		// the reference's function where oracle/_ref was built, beside this binary's tree
		char path[4096];
		const char *slash = strrchr(argv[0], '/');
		snprintf(path, sizeof(path), "%.*s/../../oracle/_ref/libcsum_ref.so", slash ? (int)(slash - argv[0]) : 1,
		         slash ? argv[0] : ".");
		void *h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
		void (*set)(int, int, unsigned) = h ? (void (*)(int, int, unsigned))dlsym(h, "ref_set_options") : NULL;
		xsknf_packet_processor_fn ref = h ? (xsknf_packet_processor_fn)dlsym(h, "xsknf_packet_processor") : NULL;
		if (set && ref) {
			set(iterations, action_drop, 1);
			xsknf_set_packet_processor(ref);
			nf = "reference";
		} else {
			xsknf_set_packet_processor(oracle_nf_packet_processor);
		}
	}
	// worker on the first CPU of our set, generators on the next ones
	cpu_set_t set;
	pthread_getaffinity_np(pthread_self(), sizeof(set), &set);
	int cpus[CPU_SETSIZE], ncpu = 0;
	for (int c = 0; c < CPU_SETSIZE; c++)
		if (CPU_ISSET(c, &set))
			cpus[ncpu++] = c;
	if (ncpu < 2 + gen_threads) {
		printf("{\"error\": \"need %d CPUs\"}\n", 2 + gen_threads);
		return 3;
	}
	nf_cpu = cpus[0];
	if ((rc = xsknf_init(&cfg, NULL))) {
		printf("{\"error\": \"xsknf_init: %s\"}\n", strerror(-rc));
		return 3;
	}
	if ((rc = xsknf_start_workers())) {
		printf("{\"error\": \"start: %s\"}\n", strerror(-rc));
		xsknf_cleanup();
		return 3;
	}
	pin_self(cpus[ncpu - 1]);

	if (check_out) {
		unsigned long got = 0;
		rc = capture(check_out, 20.0, &got);
		const int werr = xsknf_worker_error(0);
		struct xsknf_socket_stats st;
		xsknf_get_socket_stats(0, 0, &st);
		xsknf_cleanup();
		printf("{\"mode\": \"check\", \"nf\": \"%s\", \"sent\": %u, \"returned\": %lu, \"rx_npkts\": %lu, "
		       "\"tx_npkts\": %lu, \"rx_dropped\": %lu, \"tx_invalid\": %lu, \"worker_error\": %d, "
		       "\"rc\": %d}\n",
		       nf, fr.n, got, st.rx_npkts, st.tx_npkts, st.rx_dropped_npkts, st.tx_invalid_npkts, werr, rc);
		return rc || werr ? 1 : 0;
	}

	pthread_t gt[8];
	struct gen_arg ga[8];
	for (int i = 0; i < gen_threads; i++) {
		ga[i].id = i;
		ga[i].cpu = cpus[1 + i];
		pthread_create(&gt[i], NULL, generator, &ga[i]);
	}
	// warm up, then binary search (reference: MAX_LOSS 0.001, TARGET_STEP)
	unsigned long s, r;
	double ach;
	trial(0.2e6, 0.5, &s, &r, &ach);
	// a trial passes when the generators really offered the target (>= 97 %)
	// and loss <= 0.1 %; when they cannot reach it the result is generator-bound
	double lo = 0, hi = max_mpps, cur = max_mpps, best = 0, best_ach = 0, top_ach = 0, top_loss = 0;
	int trials = 0, gen_bound = 0;
	while (hi - lo > step_mpps) {
		const double loss = trial(cur * 1e6, trial_s, &s, &r, &ach);
		trials++;
		if (trials == 1) {
			top_ach = ach;
			top_loss = loss;
		}
		fprintf(stderr, "target %.3f Mpps: sent %lu (%.3f Mpps) rx %lu loss %.4f%%\n", cur, s,
			ach / 1e6, r, loss * 100);
		const int offered = ach >= 0.97 * cur * 1e6;
		if (loss <= 0.001 && offered) {
			best = cur;
			best_ach = ach;
			lo = cur;
		} else {
			if (loss <= 0.001 && ach > best_ach) {
				gen_bound = 1;     // no loss, but the target was not reached
				best_ach = ach;
				best = ach / 1e6;
			}
			hi = cur;
		}
		cur = (hi + lo) / 2;
	}
	gen_stop = 1;
	for (int i = 0; i < gen_threads; i++)
		pthread_join(gt[i], NULL);
	const int werr = xsknf_worker_error(0);
	struct xsknf_socket_stats st;
	xsknf_get_socket_stats(0, 0, &st);
	xsknf_cleanup();
	printf("{\"mode\": \"search\", \"nf\": \"%s\", \"zero_loss_mpps\": %.4f, \"achieved_mpps\": %.4f, "
	       "\"generator_bound\": %s, "
	       "\"offered_at_max_mpps\": %.4f, \"loss_at_max\": %.5f, \"trials\": %d, "
	       "\"generators\": %d, \"nf_cpu\": %d, \"iterations\": %d, \"batch\": %d, "
	       "\"rx_npkts\": %lu, \"rx_dropped\": %lu, \"rx_full\": %lu, \"fill_empty\": %lu, "
	       "\"worker_error\": %d}\n",
	       nf, best, best_ach / 1e6, gen_bound ? "true" : "false", top_ach / 1e6, top_loss, trials, gen_threads, nf_cpu, iterations,
	       batch, st.rx_npkts, st.rx_dropped_npkts, st.rx_full_npkts, st.rx_fill_empty_npkts, werr);
	return werr ? 1 : 0;
}
