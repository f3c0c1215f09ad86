"""Node configuration: a ``key = value`` settings file and a server list.

Reference: src/conf/headers/Configuration.h (defaults: 64 MiB pages, 200 connections, page header size,
shuffle / broadcast / hash page sizes, shared-memory pool, threads, batch size) read from conf/pdbSettings.conf
(``# comments``, ``key = value`` lines), and conf/serverlist (one worker address per line) used by the cluster
start scripts.

MI355X-native additions next to the reference's keys: the device (HBM) budget of the page pool, the pinned host
tier that replaces the shared-memory pool as the spill target, the broadcast-join threshold and the fusion switch.
Unknown keys are kept (``extra``) so a reference settings file loads unchanged.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field, fields
from typing import Dict, List, Optional, Tuple

MiB = 1 << 20


@dataclass
class Configuration:
    # reference keys (Configuration.h / pdbSettings.conf)
    port: int = 8108
    server_name: str = "netsdb_amd"
    my_ip: str = "127.0.0.1"
    enable_storage: bool = True
    enable_catalog: bool = True
    enable_dm: bool = True
    max_connections: int = 200
    log_file: str = "PDBserver-log"
    page_size: int = 64 * MiB
    max_page_size: int = 1024 * MiB
    shuffle_page_size: int = 1024 * MiB
    broadcast_page_size: int = 1024 * MiB
    hash_page_size: int = 512 * MiB
    shared_mem_size: Optional[int] = None      # pinned host spill tier bytes (None: 1/8 of host RAM, <= 64 GiB)
    num_threads: int = 2
    batch_size: int = 1
    root_directory: str = "netsdb_data"
    # MI355X-native keys
    device_budget: Optional[int] = None        # HBM bytes the page pool may hold before spilling (None: no cap)
    broadcast_threshold: int = 2 << 30         # joins whose build side is smaller are broadcast
    fusion: bool = True                        # tensor-pattern fusion of UDF graphs onto MFMA kernels
    extra: Dict[str, str] = field(default_factory=dict)

    # the settings file's camelCase spellings
    _ALIASES = {"port": "port", "servername": "server_name", "myip": "my_ip", "enablestorage": "enable_storage",
                "enablecatalog": "enable_catalog", "enabledm": "enable_dm", "maxconnections": "max_connections",
                "logfile": "log_file", "pagesize": "page_size", "maxpagesize": "max_page_size",
                "shufflepagesize": "shuffle_page_size", "broadcastpagesize": "broadcast_page_size",
                "hashpagesize": "hash_page_size", "sharedmemsize": "shared_mem_size", "numthreads": "num_threads",
                "batchsize": "batch_size", "rootdirectory": "root_directory", "devicebudget": "device_budget",
                "broadcastthreshold": "broadcast_threshold", "fusion": "fusion"}

    @property
    def net_page_size(self) -> int:
        """Usable bytes of a page after its header (Configuration::getNetPageSize)."""
        return self.page_size - PAGE_HEADER_SIZE

    @classmethod
    def load(cls, path: str) -> "Configuration":
        with open(path) as f:
            return cls.parse(f.read())

    @classmethod
    def parse(cls, text: str) -> "Configuration":
        conf = cls()
        types = {f.name: f.type for f in fields(cls)}
        for ln, raw in enumerate(text.splitlines(), 1):
            line = raw.split("#", 1)[0].strip()
            if not line:
                continue
            if "=" not in line:
                raise ValueError(f"line {ln}: expected 'key = value', got {raw!r}")
            key, val = (x.strip() for x in line.split("=", 1))
            name = cls._ALIASES.get(key.replace("_", "").lower())
            if name is None:
                conf.extra[key] = val
                continue
            setattr(conf, name, _coerce(val, types[name], key))
        return conf

    def client_kwargs(self) -> dict:
        """Keyword arguments of PDBClient for this node."""
        return {"page_size": self.page_size, "device_budget": self.device_budget,
                "broadcast_threshold": self.broadcast_threshold, "fusion": self.fusion,
                "pinned_budget": self.shared_mem_size}

    def dump(self) -> str:
        out = []
        for f in fields(self):
            if f.name in ("extra",):
                continue
            v = getattr(self, f.name)
            if v is None:
                continue
            out.append(f"{f.name} = {str(v).lower() if isinstance(v, bool) else v}")
        out += [f"{k} = {v}" for k, v in self.extra.items()]
        return "\n".join(out) + "\n"


# bytes reserved per page for its header (ids of node / database / type / set / page + object and reference
# counts, as Configuration.h's DEFAULT_PAGE_HEADER_SIZE reserves)
PAGE_HEADER_SIZE = 8 * 7


def _coerce(val: str, typ, key: str):
    t = str(typ)
    if "bool" in t:
        v = val.lower()
        if v in ("true", "y", "yes", "1", "on"):
            return True
        if v in ("false", "n", "no", "0", "off"):
            return False
        raise ValueError(f"{key}: expected a boolean, got {val!r}")
    if "int" in t:
        if val.lower() in ("none", ""):
            return None
        return int(val.replace("_", ""), 0)
    return val


def load_serverlist(path: str, default_port: int = 8108) -> List[Tuple[str, int]]:
    """conf/serverlist: one node per line, ``host`` or ``host:port``; ``#`` comments and blanks ignored."""
    nodes = []
    with open(path) as f:
        for raw in f:
            line = raw.split("#", 1)[0].strip()
            if not line:
                continue
            host, _, port = line.partition(":")
            nodes.append((host.strip(), int(port) if port else default_port))
    return nodes


def find_config(explicit: Optional[str] = None) -> Optional[str]:
    """The settings file to use: an explicit path, $NSDB_CONF, or ./conf/pdbSettings.conf when present."""
    for p in (explicit, os.environ.get("NSDB_CONF"), os.path.join(os.getcwd(), "conf", "pdbSettings.conf")):
        if p and os.path.exists(p):
            return p
    return None
