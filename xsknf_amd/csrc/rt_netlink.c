// rt_netlink.c -- the few rtnetlink requests the AF_XDP runtime needs, over a
// raw NETLINK_ROUTE socket (the reference uses libbpf's bpf_set_link_xdp_fd(),
// src/xsknf.c:379 / :1037, and libmnl for tc, :195-355; neither is available
// here, and only XDP attach/detach is on the checksummer's path).
//
// Also used by the test harness: veth pair creation and link up, so config 1
// (checksummer over a veth pair) can run inside a private network namespace.
#include "rt_netlink.h"

#include <errno.h>
#include <linux/if_link.h>
#include <linux/netlink.h>
#include <linux/rtnetlink.h>
#include <linux/veth.h>
#include <net/if.h>
#include <stdint.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

struct nl_req {
  struct nlmsghdr *nh;
  size_t cap;
};

static struct rtattr *nl_put(struct nl_req *r, unsigned short type, const void *data, size_t len) {
  const size_t need = NLMSG_ALIGN(r->nh->nlmsg_len) + RTA_SPACE(len);
  if (need > r->cap) return NULL;
  struct rtattr *a = (struct rtattr *)((char *)r->nh + NLMSG_ALIGN(r->nh->nlmsg_len));
  a->rta_type = type;
  a->rta_len = RTA_LENGTH(len);
  if (len) memcpy(RTA_DATA(a), data, len);
  r->nh->nlmsg_len = need;
  return a;
}

static struct rtattr *nl_nest(struct nl_req *r, unsigned short type) {
  return nl_put(r, type | NLA_F_NESTED, NULL, 0);
}

static void nl_nest_end(struct nl_req *r, struct rtattr *a) {
  a->rta_len = (unsigned short)((char *)r->nh + r->nh->nlmsg_len - (char *)a);
}

// send one request and wait for its ACK; returns 0 or -errno from the kernel
static int nl_transact(struct nlmsghdr *nh) {
  int fd = socket(AF_NETLINK, SOCK_RAW | SOCK_CLOEXEC, NETLINK_ROUTE);
  if (fd < 0) return -errno;
  struct sockaddr_nl sa = {.nl_family = AF_NETLINK};
  int rc = 0;
  nh->nlmsg_flags |= NLM_F_REQUEST | NLM_F_ACK;
  nh->nlmsg_seq = 1;
  if (sendto(fd, nh, nh->nlmsg_len, 0, (struct sockaddr *)&sa, sizeof(sa)) < 0) {
    rc = -errno;
    goto out;
  }
  for (;;) {
    char buf[4096] __attribute__((aligned(4)));
    ssize_t n = recv(fd, buf, sizeof(buf), 0);
    if (n < 0) {
      if (errno == EINTR) continue;
      rc = -errno;
      goto out;
    }
    for (struct nlmsghdr *m = (struct nlmsghdr *)buf; NLMSG_OK(m, (size_t)n); m = NLMSG_NEXT(m, n)) {
      if (m->nlmsg_type == NLMSG_ERROR) {
        const struct nlmsgerr *e = (const struct nlmsgerr *)NLMSG_DATA(m);
        rc = e->error;  // 0 = ACK
        goto out;
      }
      if (m->nlmsg_type == NLMSG_DONE) goto out;
    }
  }
out:
  close(fd);
  return rc;
}

int xsknf_nl_set_xdp(int ifindex, int prog_fd, uint32_t xdp_flags) {
  char buf[256] __attribute__((aligned(4)));
  memset(buf, 0, sizeof(buf));
  struct nl_req r = {(struct nlmsghdr *)buf, sizeof(buf)};
  r.nh->nlmsg_len = NLMSG_LENGTH(sizeof(struct ifinfomsg));
  r.nh->nlmsg_type = RTM_SETLINK;
  struct ifinfomsg *ifi = (struct ifinfomsg *)NLMSG_DATA(r.nh);
  ifi->ifi_family = AF_UNSPEC;
  ifi->ifi_index = ifindex;
  struct rtattr *x = nl_nest(&r, IFLA_XDP);
  if (!x || !nl_put(&r, IFLA_XDP_FD, &prog_fd, sizeof(prog_fd))) return -ENOBUFS;
  // only the mode bits when detaching, like a detach through libbpf
  const uint32_t f = prog_fd < 0 ? (xdp_flags & XDP_FLAGS_MODES) : xdp_flags;
  if (f && !nl_put(&r, IFLA_XDP_FLAGS, &f, sizeof(f))) return -ENOBUFS;
  nl_nest_end(&r, x);
  return nl_transact(r.nh);
}

int xsknf_nl_create_veth(const char *name, const char *peer) {
  char buf[512] __attribute__((aligned(4)));
  memset(buf, 0, sizeof(buf));
  struct nl_req r = {(struct nlmsghdr *)buf, sizeof(buf)};
  r.nh->nlmsg_len = NLMSG_LENGTH(sizeof(struct ifinfomsg));
  r.nh->nlmsg_type = RTM_NEWLINK;
  r.nh->nlmsg_flags = NLM_F_CREATE | NLM_F_EXCL;
  ((struct ifinfomsg *)NLMSG_DATA(r.nh))->ifi_family = AF_UNSPEC;
  if (!nl_put(&r, IFLA_IFNAME, name, strlen(name) + 1)) return -ENOBUFS;
  struct rtattr *li = nl_nest(&r, IFLA_LINKINFO);
  if (!li || !nl_put(&r, IFLA_INFO_KIND, "veth", 5)) return -ENOBUFS;
  struct rtattr *data = nl_nest(&r, IFLA_INFO_DATA);
  struct rtattr *pe = data ? nl_nest(&r, VETH_INFO_PEER) : NULL;
  if (!pe) return -ENOBUFS;
  // VETH_INFO_PEER carries an ifinfomsg followed by the peer's attributes
  struct ifinfomsg pi = {.ifi_family = AF_UNSPEC};
  const size_t at = NLMSG_ALIGN(r.nh->nlmsg_len);
  if (at + NLMSG_ALIGN(sizeof(pi)) > r.cap) return -ENOBUFS;
  memcpy((char *)r.nh + at, &pi, sizeof(pi));
  r.nh->nlmsg_len = at + NLMSG_ALIGN(sizeof(pi));
  if (!nl_put(&r, IFLA_IFNAME, peer, strlen(peer) + 1)) return -ENOBUFS;
  nl_nest_end(&r, pe);
  nl_nest_end(&r, data);
  nl_nest_end(&r, li);
  return nl_transact(r.nh);
}

int xsknf_nl_link_up(int ifindex) {
  char buf[128] __attribute__((aligned(4)));
  memset(buf, 0, sizeof(buf));
  struct nlmsghdr *nh = (struct nlmsghdr *)buf;
  nh->nlmsg_len = NLMSG_LENGTH(sizeof(struct ifinfomsg));
  nh->nlmsg_type = RTM_NEWLINK;
  struct ifinfomsg *ifi = (struct ifinfomsg *)NLMSG_DATA(nh);
  ifi->ifi_family = AF_UNSPEC;
  ifi->ifi_index = ifindex;
  ifi->ifi_flags = IFF_UP;
  ifi->ifi_change = IFF_UP;
  return nl_transact(nh);
}
