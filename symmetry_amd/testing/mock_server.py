"""A Symmetry server: provider registry, challenge signing, liveness, model-based assignment.

The reference ships only the provider; the server is implied by its protocol
(``src/constants.ts:3-20``) and the server-side shapes in ``src/types.ts:182-208``
(``Session``, ``PeerSessionRequest``, ``PeerWithSession``, ``PeerUpsert``) and
by the README flow (``readme.md:105-110``): providers connect, prove the
server's identity with a signed challenge, register (``join``); clients
``requestProvider`` by model and get ``providerDetails`` (the provider's
discovery key); the server balances load across providers of a model
(``readme.md:123``).  Registry rows live in SQLite (the reference lists
``sqlite3`` as a dependency and ``.gitignore``s ``sqlite.db``).

Also the fault-injection hooks used by the integration tests: ``sign_bad``
(forged signature), ``ping_interval``, ``drop_providers()``.
"""
from __future__ import annotations

import asyncio
import base64
import sqlite3
import time
import uuid

from ..net import identity
from ..net.swarm import Swarm
from ..protocol.codec import create_message, from_buffer_json, safe_parse_json
from ..protocol.keys import Keys


class SymmetryServer:
    def __init__(self, seed: bytes | None = None, bootstrap=None, ping_interval: float = 5.0, sign_bad: bool = False,
                 session_ttl: float = 3600.0):
        self.kp = identity.key_pair(seed)
        self.server_key = self.kp.public_key.hex()
        self.bootstrap = bootstrap
        self.ping_interval = ping_interval
        self.sign_bad = sign_bad
        self.session_ttl = session_ttl
        self.db = sqlite3.connect(":memory:")
        self.db.execute("CREATE TABLE providers (peer_key TEXT PRIMARY KEY, discovery_key TEXT, model_name TEXT, "
                        "public INTEGER, data_collection INTEGER, max_connections INTEGER, name TEXT, "
                        "joined REAL, last_pong REAL, assigned INTEGER DEFAULT 0, completions INTEGER DEFAULT 0)")
        self.db.execute("CREATE TABLE sessions (id TEXT PRIMARY KEY, provider_id TEXT, created REAL, expires REAL)")
        self.swarm: Swarm | None = None
        self.provider_peers: dict[str, object] = {}
        self.joins: list[dict] = []
        self.leaves: list[dict] = []
        self.challenges_signed = 0
        self.pongs = 0
        self._ping_task: asyncio.Task | None = None

    @property
    def topic(self) -> bytes:
        return identity.server_topic(self.server_key)

    async def start(self) -> None:
        # the server is every client's and provider's first hop: no small peer cap (Swarm's default is 64)
        self.swarm = Swarm(self.kp, bootstrap=self.bootstrap, max_peers=4096)
        self.swarm.on("connection", self._on_connection)
        await self.swarm.join(self.topic, server=True, client=False).flushed()
        self._ping_task = asyncio.ensure_future(self._pinger())

    async def stop(self) -> None:
        if self._ping_task:
            self._ping_task.cancel()
        if self.swarm:
            await self.swarm.destroy()

    async def _pinger(self) -> None:
        while True:
            await asyncio.sleep(self.ping_interval)
            for peer in list(self.provider_peers.values()):
                if peer.writable:
                    peer.write(create_message(Keys.PING))

    # ------------------------------------------------------------------------------------------
    def providers(self, model: str | None = None) -> list[dict]:
        cur = self.db.execute("SELECT peer_key, discovery_key, model_name, data_collection, assigned, name "
                              "FROM providers" + (" WHERE model_name = ?" if model else ""),
                              (model,) if model else ())
        return [dict(zip(("peer_key", "discovery_key", "model_name", "data_collection", "assigned", "name"), r))
                for r in cur.fetchall()]

    def _on_connection(self, peer, info=None) -> None:
        key = peer.remote_public_key.hex()

        def on_data(buf: bytes) -> None:
            msg = safe_parse_json(buf)
            if not isinstance(msg, dict):
                return
            k, data = msg.get("key"), msg.get("data")
            if k == Keys.CHALLENGE:
                ch = from_buffer_json((data or {}).get("challenge"))
                if ch is None:
                    return
                sig = identity.sign(ch, self.kp.secret_key)
                if self.sign_bad:
                    sig = bytes(64)
                self.challenges_signed += 1
                peer.write(create_message(Keys.CHALLENGE, {"message": "challenge response",
                                                           "signature": {"data": base64.b64encode(sig).decode()}}))
            elif k == Keys.JOIN:
                self._register(key, peer, data or {})
            elif k == Keys.PONG:
                self.pongs += 1
                self.db.execute("UPDATE providers SET last_pong = ? WHERE peer_key = ?", (time.time(), key))
            elif k == Keys.REQUEST_PROVIDER:
                self._assign(peer, data or {})
            elif k == Keys.VERIFY_SESSION:
                self._verify_session(peer, data or {})
            elif k == Keys.REPORT_COMPLETION:
                pid = (data or {}).get("providerId")
                self.db.execute("UPDATE providers SET completions = completions + 1 WHERE peer_key = ?", (pid,))
            elif k == Keys.LEAVE:
                self.leaves.append({"peer_key": key, "data": data})
                self._unregister(key)

        peer.on("data", on_data)
        peer.on("close", lambda: self._unregister(key))

    def _register(self, key: str, peer, cfg: dict) -> None:
        self.joins.append(cfg)
        self.provider_peers[key] = peer
        self.db.execute(
            "INSERT OR REPLACE INTO providers (peer_key, discovery_key, model_name, public, data_collection, "
            "max_connections, name, joined, last_pong) VALUES (?,?,?,?,?,?,?,?,?)",
            (key, cfg.get("discoveryKey"), cfg.get("modelName"), int(bool(cfg.get("public"))),
             int(bool(cfg.get("dataCollectionEnabled"))), int(cfg.get("maxConnections") or 0), cfg.get("name"),
             time.time(), time.time()))
        peer.write(create_message(Keys.JOIN_ACK, {"providerId": key}))

    def _unregister(self, key: str) -> None:
        self.provider_peers.pop(key, None)
        self.db.execute("DELETE FROM providers WHERE peer_key = ?", (key,))

    def _assign(self, peer, req: dict) -> None:
        model = req.get("modelName")
        preferred = req.get("preferredProviderId")
        rows = self.providers(model)
        if preferred:
            rows = [r for r in rows if r["peer_key"] == preferred] or rows
        if not rows:
            peer.write(create_message(Keys.PROVIDER_DETAILS, {"error": f"no provider for model {model!r}"}))
            return
        best = min(rows, key=lambda r: r["assigned"])  # Balance: least-assigned provider of the model
        self.db.execute("UPDATE providers SET assigned = assigned + 1 WHERE peer_key = ?", (best["peer_key"],))
        sid = str(uuid.uuid4())
        now = time.time()
        self.db.execute("INSERT INTO sessions VALUES (?,?,?,?)", (sid, best["peer_key"], now, now + self.session_ttl))
        peer.write(create_message(Keys.PROVIDER_DETAILS, {
            "providerId": best["peer_key"], "discoveryKey": best["discovery_key"], "modelName": best["model_name"],
            "dataCollectionEnabled": bool(best["data_collection"]), "sessionToken": sid}))

    def _verify_session(self, peer, req: dict) -> None:
        row = self.db.execute("SELECT provider_id, expires FROM sessions WHERE id = ?",
                              (req.get("sessionToken"),)).fetchone()
        valid = row is not None and row[1] > time.time()
        peer.write(create_message(Keys.SESSION_VALID, {"valid": valid, "providerId": row[0] if row else None}))

    def drop_providers(self) -> None:
        for peer in list(self.provider_peers.values()):
            peer.destroy()
