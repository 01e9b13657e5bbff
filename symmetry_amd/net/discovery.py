"""Topic discovery: a bootstrap registry node (the DHT analogue) and its client.

REF: hyperdht 6.15.4 / dht-rpc 6.11.3 announce a topic (32-byte discovery
key) and look up its announcers over a public Kademlia DHT
(package-lock.json:3416, :2513).  The GPU boxes have no
network, so discovery is a small registry node with the same two verbs --
announce (server mode) and lookup (client mode) -- reached over TCP on
127.0.0.1 or a LAN address.  Entries carry the announcer's ed25519 public key,
which the swarm checks against the key proven in the Noise handshake, and
expire unless refreshed (the DHT's record TTL).

Wire format: one JSON object per line.
  {"op":"announce","topic":hex,"publicKey":hex,"host":h,"port":p,"ttl":s} -> {"ok":true}
  {"op":"unannounce","topic":hex,"publicKey":hex}                       -> {"ok":true}
  {"op":"lookup","topic":hex}                                           -> {"ok":true,"peers":[...]}
"""
from __future__ import annotations

import asyncio
import json
import time

DEFAULT_TTL = 30.0


class DiscoveryServer:
    def __init__(self, host: str = "127.0.0.1", port: int = 0):
        self.host, self.port = host, port
        self.records: dict[str, dict[str, dict]] = {}
        self._server: asyncio.AbstractServer | None = None

    async def start(self) -> int:
        self._server = await asyncio.start_server(self._client, self.host, self.port)
        self.port = self._server.sockets[0].getsockname()[1]
        return self.port

    async def stop(self) -> None:
        if self._server is not None:
            self._server.close()
            await self._server.wait_closed()

    @property
    def address(self) -> tuple[str, int]:
        return self.host, self.port

    def _peers(self, topic: str) -> list[dict]:
        now = time.monotonic()
        recs = self.records.get(topic, {})
        for k in [k for k, r in recs.items() if r["expires"] < now]:
            del recs[k]
        return [{"publicKey": r["publicKey"], "host": r["host"], "port": r["port"]} for r in recs.values()]

    def handle(self, req: dict) -> dict:
        op = req.get("op")
        topic = str(req.get("topic", ""))
        if op == "announce":
            pk = str(req["publicKey"])
            ttl = float(req.get("ttl", DEFAULT_TTL))
            self.records.setdefault(topic, {})[pk] = {
                "publicKey": pk, "host": str(req["host"]), "port": int(req["port"]),
                "expires": time.monotonic() + ttl}
            return {"ok": True}
        if op == "unannounce":
            self.records.get(topic, {}).pop(str(req.get("publicKey")), None)
            return {"ok": True}
        if op == "lookup":
            return {"ok": True, "peers": self._peers(topic)}
        return {"ok": False, "error": f"unknown op {op!r}"}

    async def _client(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        try:
            while True:
                line = await reader.readline()
                if not line:
                    break
                try:
                    req = json.loads(line)
                    resp = self.handle(req)
                    if "id" in req:
                        resp["id"] = req["id"]
                except Exception as exc:  # malformed request: answer, keep serving
                    resp = {"ok": False, "error": str(exc)}
                writer.write((json.dumps(resp) + "\n").encode())
                await writer.drain()
        except (ConnectionError, asyncio.IncompleteReadError):
            pass
        finally:
            writer.close()


class DiscoveryClient:
    """Talks to one or more bootstrap nodes; results are merged."""

    def __init__(self, bootstrap: list[tuple[str, int]], timeout: float = 5.0):
        self.bootstrap = [(h, int(p)) for h, p in bootstrap]
        self.timeout = timeout
        self._conns: dict[tuple, tuple] = {}
        self._lock = asyncio.Lock()
        self._next = 0

    async def _request(self, node, req: dict) -> dict:
        async with self._lock:
            conn = self._conns.get(node)
            if conn is None or conn[1].is_closing():
                conn = await asyncio.wait_for(asyncio.open_connection(*node), self.timeout)
                self._conns[node] = conn
            reader, writer = conn
            self._next += 1
            req = dict(req, id=self._next)
            try:
                writer.write((json.dumps(req) + "\n").encode())
                await writer.drain()
                line = await asyncio.wait_for(reader.readline(), self.timeout)
            except Exception:
                self._conns.pop(node, None)
                writer.close()
                raise
            if not line:
                self._conns.pop(node, None)
                raise ConnectionError("bootstrap node closed the connection")
            return json.loads(line)

    async def _all(self, req: dict) -> list[dict]:
        out = []
        for node in self.bootstrap:
            try:
                out.append(await self._request(node, req))
            except (OSError, asyncio.TimeoutError, ConnectionError):
                continue
        return out

    async def announce(self, topic: bytes, public_key: bytes, host: str, port: int, ttl: float = DEFAULT_TTL) -> bool:
        res = await self._all({"op": "announce", "topic": topic.hex(), "publicKey": public_key.hex(), "host": host,
                               "port": port, "ttl": ttl})
        return any(r.get("ok") for r in res)

    async def unannounce(self, topic: bytes, public_key: bytes) -> None:
        await self._all({"op": "unannounce", "topic": topic.hex(), "publicKey": public_key.hex()})

    async def lookup(self, topic: bytes) -> list[dict]:
        seen, out = set(), []
        for r in await self._all({"op": "lookup", "topic": topic.hex()}):
            for p in r.get("peers", []):
                if p["publicKey"] not in seen:
                    seen.add(p["publicKey"])
                    out.append(p)
        return out

    async def close(self) -> None:
        for _, w in self._conns.values():
            w.close()
        self._conns.clear()


def main(argv=None) -> int:
    """``symmetry-dht``: run a standalone bootstrap/discovery node."""
    import argparse

    ap = argparse.ArgumentParser(prog="symmetry-dht")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=49737)
    args = ap.parse_args(argv)

    async def run():
        srv = DiscoveryServer(args.host, args.port)
        port = await srv.start()
        print(f"discovery node listening on {args.host}:{port}", flush=True)
        await asyncio.Event().wait()

    try:
        asyncio.run(run())
    except KeyboardInterrupt:
        pass
    return 0
