"""P2P plane: identities, topic discovery and the encrypted swarm transport.

The C++ data plane lives in ``csrc/net`` and is loaded as
``symmetry_amd.net._native`` (built by ``python -m symmetry_amd._build net``).
"""
from .identity import (KeyPair, discovery_key, key_pair, random_bytes, seed_from_name, server_public_key,
                       server_topic, sign, verify)

__all__ = ["KeyPair", "discovery_key", "key_pair", "random_bytes", "seed_from_name", "server_public_key",
           "server_topic", "sign", "verify", "Swarm", "DiscoveryServer", "DiscoveryClient"]


def __getattr__(name):
    if name == "Swarm":
        from .swarm import Swarm
        return Swarm
    if name in ("DiscoveryServer", "DiscoveryClient"):
        from . import discovery
        return getattr(discovery, name)
    raise AttributeError(name)
