"""Node configuration (utils/config.py; reference src/conf Configuration.h + conf/pdbSettings.conf, serverlist)."""
import os

import pytest

from netsdb_amd.utils.config import Configuration, find_config, load_serverlist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_parse_reference_style_settings():
    text = """
    # comment
    port = 9000
    serverName =testServer
    enableStorage=true
    useUnixDomainSock=false
    maxConnections=100
    pageSize=65536   # trailing comment
    sharedMemSize = 805306368
    deviceBudget = 1_000_000
    fusion = n
    """
    c = Configuration.parse(text)
    assert (c.port, c.server_name, c.enable_storage, c.max_connections) == (9000, "testServer", True, 100)
    assert c.page_size == 65536 and c.net_page_size == 65536 - 56
    assert c.shared_mem_size == 805306368 and c.device_budget == 1_000_000 and c.fusion is False
    assert c.extra == {"useUnixDomainSock": "false"}
    assert Configuration.parse(c.dump()).page_size == 65536
    with pytest.raises(ValueError):
        Configuration.parse("fusion = maybe")
    with pytest.raises(ValueError):
        Configuration.parse("just a line")


def test_shipped_conf_and_serverlist(tmp_path):
    c = Configuration.load(os.path.join(ROOT, "conf", "pdbSettings.conf"))
    assert c.page_size == 64 << 20 and c.port == 8108 and c.fusion is True
    assert load_serverlist(os.path.join(ROOT, "conf", "serverlist")) == [("127.0.0.1", 8108)]
    p = tmp_path / "servers"
    p.write_text("10.0.0.1\n10.0.0.2:9000  # worker\n\n")
    assert load_serverlist(str(p)) == [("10.0.0.1", 8108), ("10.0.0.2", 9000)]
    assert find_config(str(p)) == str(p)


def test_client_from_config(tmp_path):
    from netsdb_amd.client import PDBClient

    p = tmp_path / "s.conf"
    p.write_text(f"pageSize = 131072\nbroadcastThreshold = 0\nrootDirectory = {tmp_path / 'data'}\n")
    c = PDBClient.from_config(str(p))
    assert c.storage.page_size == 131072 and c.engine.broadcast_threshold == 0
