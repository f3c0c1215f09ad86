"""Home-tier page arena (storage/devpool.py): page columns carved out of arena chunks by the native slab
allocator (reference src/memory SlabAllocator + src/bufferMgr page pool) — allocation, reuse after free,
coalescing, spill/reload and set removal returning regions, and a GPU run with HBM eviction."""
import pytest
import torch

from netsdb_amd.client import PDBClient
from netsdb_amd.objects.record import RecordBatch
from netsdb_amd.storage.devpool import DevicePagePool


def test_pool_alloc_free_coalesce_cpu():
    pool = DevicePagePool("cpu", chunk_bytes=1 << 20)
    a = pool.alloc(1000)
    b = pool.alloc(300_000)
    c = pool.alloc(800_000)          # no room left in chunk 0 -> a second chunk
    assert pool.stats["chunks"] == 2 and a[0] == 0 and b[0] == 0 and c[0] == 1
    v = pool.view(b, torch.float32, (75_000,))
    v.fill_(3.0)
    assert pool.view(b, torch.float32, (75_000,)).sum().item() == 225_000.0
    pool.release([a, b])
    assert pool.slabs[0].used == 0 and pool.slabs[0].largest_free == 1 << 20    # neighbours coalesced
    d = pool.alloc(1 << 20)          # the whole first chunk again
    assert d == (0, 0)


def test_pages_live_in_the_arena_and_return_on_remove(tmp_path):
    c = PDBClient(root=str(tmp_path), device="cpu")
    c.create_database("db")
    c.create_set("db", "s", type_=None)
    st = c.storage
    pool = st.page_pool
    assert pool is not None
    x = torch.arange(200_000, dtype=torch.float32)
    st.get_set("db", "s").add_batch(RecordBatch({"x": x, "y": x.to(torch.int64)}, 200_000))
    used = pool.used()
    assert used >= x.numel() * 12
    pages = st.get_set("db", "s").pages
    assert all(p.regions for p in pages)
    base = pool.arenas[0].data_ptr()
    col = pages[0].batch.columns["x"]
    assert base <= col.data_ptr() < base + pool.arenas[0].numel()     # a view into the arena
    got = torch.cat([b.columns["x"] for b in st.get_set("db", "s").scan()])
    torch.testing.assert_close(got, x)
    st.remove_set("db", "s")
    assert pool.used() > 0            # `col` and `got`'s sources: a held view keeps its region
    del col, pages
    assert pool.used() == 0 and pool.stats["frees"] >= pool.stats["allocs"] - 0


def test_spill_and_reload_release_and_readopt(tmp_path):
    c = PDBClient(root=str(tmp_path), device="cpu")
    st = c.storage
    c.create_database("db")
    c.create_set("db", "s", type_=None)
    s = st.get_set("db", "s")
    x = torch.randn(50_000)
    s.add_batch(RecordBatch({"x": x}, 50_000))
    p = s.pages[0]
    used = st.page_pool.used()
    assert used > 0
    freed = p.spill()
    assert freed > 0 and p.regions == [] and st.page_pool.used() == 0
    b = p.load("cpu")
    assert p.regions and st.page_pool.used() == used
    torch.testing.assert_close(b.columns["x"], x)


@pytest.mark.gpu
def test_gpu_pages_in_hbm_arena_with_eviction(tmp_path):
    c = PDBClient(root=str(tmp_path), device="cuda:0")
    st = c.storage
    st.device_budget = 64 << 20               # force evictions (to the pinned tier) and reloads
    c.create_database("db")
    c.create_set("db", "s", type_=None)
    s = st.get_set("db", "s")
    xs = [torch.randn(4 << 20) for _ in range(6)]       # 6 x 16 MiB host records: H2D straight into the arena
    for x in xs:
        s.add_batch(RecordBatch({"x": x}, x.numel()))
    assert st.stats["evicted_pages"] > 0
    assert st.page_pool.stats["allocs"] >= 6 and st.page_pool.is_cuda
    resident = [p for p in s.pages if p.location == "device"]
    assert resident and all(p.regions for p in resident)
    got = [b.columns["x"] for b in s.scan()]          # evicted pages come back into arena regions
    assert all(p.regions for p in s.pages if p.location == "device")
    for g, x in zip(got, xs):
        assert g.is_cuda
        torch.testing.assert_close(g.cpu(), x)
    # a page a device kernel produced is kept as is (no extra device copy)
    y = torch.randn(1000, device="cuda:0")
    s.add_batch(RecordBatch({"x": y}, 1000))
    assert s.pages[-1].regions == [] and s.pages[-1].batch.columns["x"].data_ptr() == y.data_ptr()
    st.remove_set("db", "s")
    torch.cuda.synchronize()
    st.page_pool._reclaim(block=True)
    assert st.page_pool.used() > 0            # `got` still views reloaded pages: their regions stay
    del got, g
    torch.cuda.synchronize()
    st.page_pool._reclaim(block=True)
    assert st.page_pool.used() == 0


def test_held_batches_survive_spill_and_region_reuse(tmp_path):
    """A batch yielded by scan() stays valid after its page is spilled and the arena region is reused by the
    next page load (the region is freed with the last tensor viewing it, not with page residency)."""
    c = PDBClient(root=str(tmp_path), device="cpu")
    st = c.storage
    st.device_budget = 17 << 20
    c.create_database("db")
    s = st.create_set("db", "s", page_size=4 << 20)
    x = torch.arange(10_000_000, dtype=torch.float32)
    s.add_batch(RecordBatch({"x": x}, x.numel()))
    assert st.stats["evicted_pages"] > 0
    held = [b.columns["x"][1:] for b in s.scan()]     # derived views only: the page batches themselves are dropped
    got = torch.cat([torch.cat([x[:1] * 0, h]) for h in held])
    starts = torch.tensor([0] + [h.numel() + 1 for h in held]).cumsum(0)[:-1]
    ref = x.clone()
    ref[starts] = 0
    torch.testing.assert_close(got, ref)
    torch.testing.assert_close(s.all().columns["x"], x)


def test_chunks_without_live_regions_go_back(tmp_path):
    pool = DevicePagePool("cpu", chunk_bytes=1 << 20)
    regs = [pool.alloc_region(600_000) for _ in range(4)]     # one region per chunk
    assert pool.stats["chunks"] == 4
    keep = regs[0].tensor()[:10]                               # a view keeps region 0 (and chunk 0) alive
    del regs
    assert pool.used() >= 600_000 and len(pool.slabs) == 1
    assert pool.stats["chunks_released"] == 3
    del keep
    assert pool.used() == 0


def test_dense_panel_spill_with_large_pool_pages(tmp_path):
    """Dense spill slabs use a spill set of their own with page numbers from 0: a panel larger than the pool
    spills with 64 MiB pages (page_no * page_size stays far below the file-size limit)."""
    from netsdb_amd.storage.manager import StorageManager

    st = StorageManager(root=str(tmp_path), device=None, page_size=64 << 20, pool_pages=2)
    d = st.create_set("db", "m", dense=True)
    panel = torch.randn(3 * 1024, 8192 * 2)                   # 192 MiB f32 > 2 pool pages of 64 MiB
    d.set_panel(panel.clone(), 3 * 1024, 8192 * 2, 1024, 1024)
    freed = d.spill()
    assert freed > 0 and d.is_spilled()
    torch.testing.assert_close(d.panel, panel)
    st.remove_set("db", "m")
