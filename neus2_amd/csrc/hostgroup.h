// Cross-process host-staged collectives over TCP (NeusHostGroup, include/neus2_hip.h neus_host_group_create).
//
// The data-parallel step issues its all-reduces through one interface; RCCL carries them between GPUs. This
// backend carries the same collectives between processes that cannot form an RCCL communicator - several ranks on one
// GPU (RCCL refuses duplicate devices), or bring-up on hosts without a working xGMI fabric - so that the product's
// multi-process path (spawned ranks, rendezvous, comm-stream overlap) runs end to end anywhere. Each collective is staged
// on the testbed's communication stream: a device-to-host copy into a pinned buffer, a host function (hipLaunchHostFunc)
// that exchanges the buffer over the sockets, a host-to-device copy back; the stream order gates it by the same events as
// the RCCL collectives and the step's stream keeps running beside it.
//
// Topology: a star through rank 0. Every other rank sends {header, payload}; rank 0 checks that every rank issued the same
// collective (sequence number, size, type, op: a mismatch - e.g. ranks with different exchange settings - fails loudly
// instead of pairing the wrong buffers), reduces in rank order (v0 + v1 + ... as NeusLocalGroup, so the result is bitwise
// the in-process group's), and sends the result back. A host-function failure cannot throw through the HIP runtime: it
// poisons the group (sockets shut down, so the peers fail too) and the next step boundary raises.
//
// Joining: every rank's hello carries {magic, rank, job token}. The token is a per-job 64-bit value the launcher hands
// every rank (bench.py draws it at random on rank 0 and broadcasts it with the port); rank 0 drops a connection whose
// hello is malformed, carries another token or names a rank already joined, and keeps waiting for the real ranks. The
// token is a guard against stray or foreign connections, not authentication against an attacker who can read the
// launcher's traffic: the default address is 127.0.0.1, and a non-loopback address exposes the port to its network.
#pragma once

#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

struct NeusHostGroup {
	enum Op : uint32_t { SUM = 0, MAX = 1 };
	enum Type : uint32_t { F32 = 0, U32 = 1 };
	struct Header { uint32_t magic, op, type, pad; uint64_t seq, bytes; };
	struct Hello { uint32_t magic; int32_t rank; uint64_t token; };
	static constexpr uint32_t MAGIC = 0x4e484731u;  // "NHG1"
	static constexpr int TIMEOUT_MS = 120000;
	static constexpr int HELLO_TIMEOUT_MS = 5000;    // a connection that sends no hello this long is dropped

	int rank = 0, world = 1;
	std::vector<int> fd;           // rank 0: fd[r] = socket of rank r (r >= 1); others: fd[0] = socket of rank 0
	std::vector<uint8_t> recv_buf; // rank 0: one peer's payload
	uint64_t seq = 0;              // collectives executed (host-function order = issue order: one stream)
	std::atomic<bool> failed{false};
	std::mutex err_mu;
	std::string err;

	NeusHostGroup(int r, int w, const char* host, int port, uint64_t token) : rank(r), world(w) {
		if (w < 1 || r < 0 || r >= w) throw std::runtime_error("host group: invalid rank / world");
		fd.assign(w, -1);
		if (w == 1) return;
		sockaddr_in addr{};
		addr.sin_family = AF_INET;
		addr.sin_port = htons((uint16_t)port);
		if (inet_pton(AF_INET, host, &addr.sin_addr) != 1) throw std::runtime_error(std::string("host group: bad address ") + host);
		if (r == 0) {
			const int ls = socket(AF_INET, SOCK_STREAM, 0);
			if (ls < 0) throw std::runtime_error("host group: socket");
			const int one = 1;
			setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
			if (bind(ls, (sockaddr*)&addr, sizeof(addr)) != 0 || listen(ls, w) != 0) {
				close(ls);
				throw std::runtime_error("host group: rank 0 cannot listen on " + std::string(host) + ":" + std::to_string(port));
			}
			const auto t0 = std::chrono::steady_clock::now();
			int joined = 0, dropped = 0;
			while (joined < w - 1) {
				const int left = TIMEOUT_MS - (int)std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
				pollfd p{ls, POLLIN, 0};
				if (left <= 0 || poll(&p, 1, left) <= 0) {
					close(ls); shutdown_all();
					throw std::runtime_error("host group: " + std::to_string(joined) + " of " + std::to_string(w - 1) + " ranks joined in time (" +
					                         std::to_string(dropped) + " connections dropped: wrong job token, rank or hello)");
				}
				const int s = accept(ls, nullptr, nullptr);
				if (s < 0) continue;
				Hello hi{};
				bool ok = true;
				try { recv_all(s, &hi, sizeof(hi), HELLO_TIMEOUT_MS); } catch (const std::exception&) { ok = false; }
				ok = ok && hi.magic == MAGIC && hi.token == token && hi.rank >= 1 && hi.rank < w && fd[hi.rank] < 0;
				if (!ok) { close(s); ++dropped; continue; }
				tune(s);
				fd[hi.rank] = s;
				++joined;
			}
			close(ls);
		} else {
			const auto t0 = std::chrono::steady_clock::now();
			int s = -1;
			for (;;) {  // rank 0 may not listen yet
				s = socket(AF_INET, SOCK_STREAM, 0);
				if (s < 0) throw std::runtime_error("host group: socket");
				if (connect(s, (sockaddr*)&addr, sizeof(addr)) == 0) break;
				close(s);
				if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(TIMEOUT_MS))
					throw std::runtime_error("host group: cannot reach rank 0 at " + std::string(host) + ":" + std::to_string(port));
				std::this_thread::sleep_for(std::chrono::milliseconds(20));
			}
			tune(s);
			const Hello me{MAGIC, r, token};
			send_all(s, &me, sizeof(me));
			fd[0] = s;
		}
	}
	~NeusHostGroup() { shutdown_all(); }

	static void tune(int s) {
		const int one = 1;
		setsockopt(s, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
	}
	void shutdown_all() {
		for (int& s : fd)
			if (s >= 0) { ::shutdown(s, SHUT_RDWR); close(s); s = -1; }
	}
	static void send_all(int s, const void* p, size_t n) {
		const uint8_t* b = (const uint8_t*)p;
		while (n) {
			pollfd q{s, POLLOUT, 0};
			if (poll(&q, 1, TIMEOUT_MS) <= 0) throw std::runtime_error("host group: send timeout");
			const ssize_t k = ::send(s, b, n, MSG_NOSIGNAL);
			if (k <= 0) throw std::runtime_error("host group: peer closed (send)");
			b += k; n -= (size_t)k;
		}
	}
	static void recv_all(int s, void* p, size_t n, int timeout_ms = TIMEOUT_MS) {
		uint8_t* b = (uint8_t*)p;
		while (n) {
			pollfd q{s, POLLIN, 0};
			if (poll(&q, 1, timeout_ms) <= 0) throw std::runtime_error("host group: receive timeout (a rank did not reach the collective)");
			const ssize_t k = ::recv(s, b, n, 0);
			if (k <= 0) throw std::runtime_error("host group: peer closed (receive)");
			b += k; n -= (size_t)k;
		}
	}
	template <class T> static void reduce(T* out, const T* v, size_t n, uint32_t op) {
		if (op == SUM) for (size_t k = 0; k < n; ++k) out[k] = (T)(out[k] + v[k]);
		else for (size_t k = 0; k < n; ++k) out[k] = out[k] < v[k] ? v[k] : out[k];
	}
	// In-place all-reduce of a host buffer (the host function's body). Rank order reduction on rank 0.
	void allreduce_host(void* buf, size_t bytes, uint32_t type, uint32_t op) {
		if (failed.load()) return;
		try {
			const Header h{MAGIC, op, type, 0u, seq++, bytes};
			if (world == 1) return;
			if (rank != 0) {
				send_all(fd[0], &h, sizeof(h));
				send_all(fd[0], buf, bytes);
				Header a{};
				recv_all(fd[0], &a, sizeof(a));
				if (a.magic != MAGIC || a.seq != h.seq || a.bytes != bytes) throw std::runtime_error("host group: reply out of step with the request");
				recv_all(fd[0], buf, bytes);
				return;
			}
			recv_buf.resize(bytes);
			for (int r = 1; r < world; ++r) {  // rank order: out = v0 + v1 + ... (NeusLocalGroup's order)
				Header a{};
				recv_all(fd[r], &a, sizeof(a));
				if (a.magic != MAGIC || a.seq != h.seq || a.bytes != h.bytes || a.op != h.op || a.type != h.type)
					throw std::runtime_error("host group: rank " + std::to_string(r) + " issued a different collective (#" + std::to_string(a.seq) + ", " +
					                         std::to_string(a.bytes) + " B) than rank 0 (#" + std::to_string(h.seq) + ", " + std::to_string(h.bytes) +
					                         " B): the ranks' step settings differ");
				recv_all(fd[r], recv_buf.data(), bytes);
				if (type == F32) reduce((float*)buf, (const float*)recv_buf.data(), bytes / 4, op);
				else reduce((uint32_t*)buf, (const uint32_t*)recv_buf.data(), bytes / 4, op);
			}
			for (int r = 1; r < world; ++r) {
				send_all(fd[r], &h, sizeof(h));
				send_all(fd[r], buf, bytes);
			}
		} catch (const std::exception& e) {
			{
				std::lock_guard<std::mutex> lk(err_mu);
				err = e.what();
			}
			failed.store(true);
			shutdown_all();  // the peers' pending receives fail instead of waiting out the timeout
		}
	}
	void check() {
		if (!failed.load()) return;
		std::lock_guard<std::mutex> lk(err_mu);
		throw std::runtime_error("data parallel (host group): " + err);
	}
};

// One staged collective's host-function argument (owned by the call; freed by the host function).
struct HostCollCall {
	NeusHostGroup* g;
	void* host;
	size_t bytes;
	uint32_t type, op;
};
