"""LMS server process: Raft node + LMS/RaftService/FileTransferService on one gRPC port.

CLI-compatible with the reference (``lms_server.py:1604-1613``)::

    python lms_server.py <id> <port> <peer_address> [<peer_address> ...]

The peers are the OTHER servers' addresses listed in server-id order, so with ids 1..N server
``id`` maps peer position k to id ``k+1`` if ``k+1 < id`` else ``k+2`` -- the real ids (the
reference keyed them 1..N-1 positionally, so server k never contacted server k+1, Appendix A.3).
Everything else (data dir, tutoring address, relevance gate, timeouts) is an optional flag.
"""
from __future__ import annotations

import argparse
import logging
import os
import signal
import threading
from concurrent import futures

import grpc

from .. import wire
from ..raft.core import RaftConfig
from ..raft.node import RaftNode
from ..raft.storage import FileStorage
from ..raft.transport import GrpcTransport, RaftServicer, snapshot_handler
from ..utils.config import parse_with_config
from ..utils.debug_rpc import debug_handler
from .blobs import BlobFetcher, BlobReplicator, fetch_handler
from .service import FileTransferServicer, LMSServicer, TutoringClient
from .state import LMSState

log = logging.getLogger("dlms.server")


def peer_ids(self_id: int, n_peers: int) -> list[int]:
    return [i for i in range(1, n_peers + 2) if i != self_id]


class LMSServer:
    def __init__(self, node_id: int, port: int, peers: dict[int, str], data_dir: str, host: str = "[::]",
                 advertise: str | None = None, tutor_address: str | None = None, gate=None,
                 raft_config: RaftConfig | None = None, fsync: bool = True, workers: int = 32,
                 snapshot_every: int = 2000, frontend: str = "aio"):
        self.id = node_id
        self.port = port
        self.peers = dict(peers)
        self.address = advertise or f"localhost:{port}"
        self.addresses = {**self.peers, node_id: self.address}
        self.data_dir = data_dir
        os.makedirs(data_dir, exist_ok=True)
        self.storage = FileStorage(os.path.join(data_dir, "raft"), fsync=fsync)
        self.state = LMSState(data_dir)
        cfg = raft_config or RaftConfig()
        self.transport = GrpcTransport(node_id, self.peers, rpc_timeout=max(cfg.rpc_timeout, 0.2))
        self.node = RaftNode(node_id, self.peers, self.storage, self.state, self.transport, cfg,
                             snapshot_every=snapshot_every)
        self.transport.attach(self.node)
        self.tutor = TutoringClient(tutor_address) if tutor_address else None
        # uploads: pushed to a majority before their (tiny) PutBlob entry is proposed; pulled from
        # a peer by any replica that missed the push (lms/blobs.py)
        self.replicator = BlobReplicator(self.state.blobs, self.peers)
        self.fetcher = BlobFetcher(self.state.blobs, self.peers, leader_id=lambda: self.node.leader_id)
        self.state.blobs.fetcher = self.fetcher
        self.lms = LMSServicer(self.node, self.state, self.addresses, tutor=self.tutor, gate=gate,
                               replicator=self.replicator)
        if gate is not None and hasattr(gate, "attach_state"):
            gate.attach_state(self.state)
        opts = [("grpc.max_send_message_length", wire.DEFAULT_MAX_MESSAGE),
                ("grpc.max_receive_message_length", wire.DEFAULT_MAX_MESSAGE)]
        self.raft_servicer = RaftServicer(self.node, self.addresses, blocked=self.transport.blocked)
        self.frontend = frontend
        self._loop = None

        def populate(server, lms):
            wire.register(server, "LMS", lms)
            wire.register(server, "RaftService", self.raft_servicer)
            wire.register(server, "FileTransferService", FileTransferServicer(self.state))
            server.add_generic_rpc_handlers((snapshot_handler(self.node), fetch_handler(self.state.blobs),
                                             debug_handler(health=self._health, status=self._status)))
            return server.add_insecure_port(f"{host}:{port}")

        if frontend == "aio":
            # grpc.aio on its own event-loop thread: the synchronous handlers (Raft RPCs, writes,
            # reads) run on the ``workers`` pool exactly as before, while GetLLMAnswer awaits the
            # tutoring tier on the loop, so in-flight tutoring queries are not capped by the pool
            import asyncio

            self._pool = futures.ThreadPoolExecutor(max_workers=workers, thread_name_prefix="lms")
            self._loop = asyncio.new_event_loop()
            self._loop.set_default_executor(self._pool)
            self._loop_thread = threading.Thread(target=self._loop.run_forever, name=f"lms{node_id}-aio",
                                                 daemon=True)
            self._loop_thread.start()

            async def make():
                srv = grpc.aio.server(migration_thread_pool=self._pool, options=opts)
                return srv, populate(srv, _AioLMSView(self.lms))

            self.server, bound = asyncio.run_coroutine_threadsafe(make(), self._loop).result(30)
        elif frontend == "threads":
            self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=workers), options=opts)
            bound = populate(self.server, self.lms)
        else:
            raise ValueError(f"unknown frontend {frontend!r}")
        if bound == 0:
            raise RuntimeError(f"could not bind {host}:{port}")
        self.port = bound

    def _health(self) -> dict:
        st = self.node.status()
        return {"node": self.id, "role": st["role"], "leader": st["leader"], "term": st["term"],
                "ok": st["leader"] is not None}

    def _status(self) -> dict:
        st = self.node.status()
        st["transport_pending"] = self.transport.pending()
        st["blobs_pushed"], st["blobs_fetched"] = self.replicator.pushed, self.fetcher.fetched
        return st

    def _on_loop(self, coro, timeout: float = 30.0):
        import asyncio

        return asyncio.run_coroutine_threadsafe(coro, self._loop).result(timeout)

    def start(self):
        if self._loop is not None:
            self._on_loop(self.server.start())
        else:
            self.server.start()
        self.node.start()
        log.info("LMS server %d listening on %s (peers %s)", self.id, self.port, self.peers)
        return self

    def stop(self, grace: float = 0.5):
        self.node.stop()
        self.transport.close()
        self.replicator.close()
        self.fetcher.close()
        if self._loop is not None:
            try:
                self._on_loop(self.server.stop(grace))
                if self.tutor is not None:
                    self._on_loop(self.tutor.aclose())
            finally:
                self._loop.call_soon_threadsafe(self._loop.stop)
                self._loop_thread.join(5)
                self._pool.shutdown(wait=False)
        else:
            self.server.stop(grace).wait()
        self.storage.close()
        if self.tutor is not None:
            self.tutor.close()

    def isolate(self, peers: set[int]):
        """Fault injection: drop all Raft traffic to/from ``peers`` (both directions)."""
        self.transport.blocked.clear()
        self.transport.blocked.update(peers)


class _AioLMSView:
    """The LMS servicer as the aio server sees it: GetLLMAnswer is the coroutine, every other
    method is the synchronous one (run on the migration thread pool)."""

    def __init__(self, servicer: LMSServicer):
        self._svc = servicer
        self.GetLLMAnswer = servicer.GetLLMAnswerAsync

    def __getattr__(self, name):
        return getattr(self._svc, name)


def cluster_from_args(args, conf: dict) -> tuple[dict[int, str], int, str | None]:
    """(peers by real id, listen port, advertised address) from the positional form
    ``<id> <port> <peers...>`` or from a config file's ``servers`` map."""
    servers = {int(k): str(v) for k, v in (conf.get("servers") or {}).items()}
    if servers and not args.peers:
        if args.id not in servers:
            raise SystemExit(f"server id {args.id} not in the config's servers {sorted(servers)}")
        port = args.port or int(servers[args.id].rsplit(":", 1)[1])
        return {i: a for i, a in servers.items() if i != args.id}, port, args.advertise or servers[args.id]
    if args.port is None:
        raise SystemExit("port required (or --config with a servers map)")
    return dict(zip(peer_ids(args.id, len(args.peers)), args.peers)), args.port, args.advertise


def build_arg_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="Raft-replicated LMS server (MI355X-native framework)")
    ap.add_argument("id", type=int, help="this server's id (1..N)")
    ap.add_argument("port", type=int, nargs="?", default=None, help="listen port (default: from --config servers)")
    ap.add_argument("peers", nargs="*", help="addresses of the other servers, in server-id order")
    ap.add_argument("--host", default="[::]")
    ap.add_argument("--advertise", default=None, help="address other nodes/clients use for this server")
    ap.add_argument("--data-dir", default=None, help="default: ./lms_node<id>")
    ap.add_argument("--tutor", default=os.environ.get("DLMS_TUTOR_ADDR", "localhost:50054"),
                    help="tutoring server address ('' to disable)")
    ap.add_argument("--gate", choices=["bert", "remote", "off"], default=os.environ.get("DLMS_GATE", "bert"),
                    help="bert: a BERT encoder in this process (GPU if visible, else CPU torch); remote: the GPU "
                         "tier's gate servers (--gate-addr), the local encoder only as --gate-fallback")
    ap.add_argument("--gate-addr", default=os.environ.get("DLMS_GATE_ADDR", ""),
                    help="gate server addresses, comma-separated (python -m distributed_lms_raft_llm_amd.gate, "
                         "or tutoring_server.py --gate-port)")
    ap.add_argument("--gate-fallback", choices=["bert", "off"], default="bert",
                    help="with --gate remote: what decides when no gate server answers (off: admit)")
    ap.add_argument("--gate-model", default="bert-base-uncased")
    ap.add_argument("--gate-device", default=os.environ.get("DLMS_GATE_DEVICE", "auto"))
    ap.add_argument("--gate-threshold", type=float, default=0.6)
    ap.add_argument("--gate-weights", default=None, help="local safetensors for the gate model")
    ap.add_argument("--vocab", default=None, help="BERT vocab.txt (WordPiece); synthetic vocab if absent")
    ap.add_argument("--election-timeout", default="0.15,0.30")
    ap.add_argument("--heartbeat", type=float, default=0.05)
    ap.add_argument("--no-fsync", action="store_true")
    ap.add_argument("--snapshot-every", type=int, default=2000)
    ap.add_argument("--workers", type=int, default=32, help="thread pool for the synchronous RPC handlers")
    ap.add_argument("--frontend", choices=("aio", "threads"), default="aio",
                    help="aio: GetLLMAnswer awaits the tutoring tier without holding a worker thread")
    ap.add_argument("--log-level", default=os.environ.get("DLMS_LOG", "INFO"))
    return ap


def main(argv=None):
    args, conf = parse_with_config(build_arg_parser(), argv)
    logging.basicConfig(level=getattr(logging, args.log_level.upper(), logging.INFO),
                        format="%(asctime)s %(name)s %(levelname)s %(message)s")
    peers, port, advertise = cluster_from_args(args, conf)
    args.port, args.advertise = port, advertise
    lo, hi = (float(x) for x in args.election_timeout.split(","))
    cfg = RaftConfig(election_timeout=(lo, hi), heartbeat_interval=args.heartbeat)
    gate = None
    if args.gate == "bert":
        from ..gate.relevance import RelevanceGate

        gate = RelevanceGate.create(model=args.gate_model, device=args.gate_device, threshold=args.gate_threshold,
                                    weights=args.gate_weights, vocab=args.vocab)
    elif args.gate == "remote":
        from ..gate.relevance import RelevanceGate
        from ..gate.service import RemoteGate

        addrs = [a.strip() for a in args.gate_addr.split(",") if a.strip()]
        if not addrs:
            raise SystemExit("--gate remote needs --gate-addr")
        fallback = None
        if args.gate_fallback == "bert":
            def fallback():
                return RelevanceGate.create(model=args.gate_model, device=args.gate_device,
                                            threshold=args.gate_threshold, weights=args.gate_weights,
                                            vocab=args.vocab)
        gate = RemoteGate(addrs, threshold=args.gate_threshold, fallback_factory=fallback)
    srv = LMSServer(args.id, args.port, peers, args.data_dir or f"lms_node{args.id}", host=args.host,
                    advertise=args.advertise, tutor_address=args.tutor or None, gate=gate, raft_config=cfg,
                    fsync=not args.no_fsync, snapshot_every=args.snapshot_every, workers=args.workers,
                    frontend=args.frontend).start()
    done = threading.Event()
    signal.signal(signal.SIGTERM, lambda *a: done.set())
    signal.signal(signal.SIGINT, lambda *a: done.set())
    done.wait()
    srv.stop()


if __name__ == "__main__":
    main()
