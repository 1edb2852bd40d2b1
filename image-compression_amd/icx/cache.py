"""L2 learned-parameter cache: the reference's H2CacheManager surface
(cache/H2CacheManager.java:23-171) on a file database.

H2 is a Java database engine and cannot be embedded here; SQLite (Python
stdlib) stands in with the same schema and the same semantics:

  * table LEARNED_PARAMS_CACHE(WIDTH_BUCKET INT, HEIGHT_BUCKET INT,
    SIZE_BUCKET BIGINT, QUALITY FLOAT, SCALE DOUBLE, PK(w, h, s))  (:48-55)
  * the configured path is made absolute and every ".mv.db" in it removed
    (`toAbsolutePath().toString().replace(".mv.db", "")`, :32); the file is
    "<path>.icx.sqlite"
  * load_all_to_map reads every row into the in-memory L1 map (:68-93); a
    database error is logged and the rows read so far are returned, so a
    corrupt or locked cache file means a cold cache, not an aborted batch
  * save_all_from_map upserts (MERGE) every entry in batches of 1000 inside
    one transaction (:100-155); on a database error the transaction is rolled
    back and the error logged (:139-152)
  * the L1 map itself is a plain dict guarded by the caller (the reference's
    ConcurrentHashMap, :69); quality values stay float32-exact.
"""
import logging
import os
import sqlite3
import threading

import numpy as np

from .core import LearnedParams, SimilarityKey

log = logging.getLogger("icx.cache")

SCHEMA = """CREATE TABLE IF NOT EXISTS LEARNED_PARAMS_CACHE (
    WIDTH_BUCKET INT NOT NULL,
    HEIGHT_BUCKET INT NOT NULL,
    SIZE_BUCKET BIGINT NOT NULL,
    QUALITY FLOAT NOT NULL,
    SCALE DOUBLE NOT NULL,
    PRIMARY KEY (WIDTH_BUCKET, HEIGHT_BUCKET, SIZE_BUCKET))"""


def db_file(path) -> str:
    return os.path.abspath(str(path)).replace(".mv.db", "") + ".icx.sqlite"


class LockedDict(dict):
    """dict with an explicit lock for compound updates (ConcurrentHashMap role)."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.lock = threading.Lock()


class SharedCache(LockedDict):
    """The L1 map shared by every rank of a multi-process run: the
    reference's one ConcurrentHashMap (CompressionBatch.java:71) when the
    file list is sharded over one process per GPU.

    Each rank keeps a local map (loaded from the same L2 file); an entry a
    rank learns is also appended to one log key in the process group's
    key-value store (the torchrun rendezvous TCPStore: 28 bytes per entry,
    no collective, ranks never wait on each other), and refresh() - called
    by the pipeline before it probes a group's keys - applies the entries
    other ranks appended since the last refresh.  Every rank applies the log
    in its order, so all converge on the same last-writer-wins map."""

    LOG = "icx/learned_cache/log"
    _REC = np.dtype([("w", "<i4"), ("h", "<i4"), ("s", "<i8"), ("q", "<f4"), ("scale", "<f8")])

    def __init__(self, store, *a, **k):
        super().__init__(*a, **k)
        self.store = store
        self._seen = 0  # bytes of the log applied so far

    def __setitem__(self, key, value):
        super().__setitem__(key, value)
        rec = np.zeros(1, self._REC)
        rec[0] = (key.width_bucket, key.height_bucket, key.size_bucket, np.float32(value.quality), value.scale)
        self.store.append(self.LOG, rec.tobytes())

    def refresh(self) -> int:
        """Apply the log's new entries (other ranks' and this rank's own, in
        log order); returns how many were read."""
        if not self.store.check([self.LOG]):
            return 0
        data = self.store.get(self.LOG)
        n = (len(data) - self._seen) // self._REC.itemsize
        if n <= 0:
            return 0
        recs = np.frombuffer(data, self._REC, n, self._seen)
        self._seen += n * self._REC.itemsize
        for r in recs:
            dict.__setitem__(self, SimilarityKey(int(r["w"]), int(r["h"]), int(r["s"])),
                             LearnedParams(float(r["q"]), float(r["scale"])))
        return n


class CacheManager:
    def __init__(self, path):
        self.path = db_file(path)
        d = os.path.dirname(os.path.abspath(self.path))
        os.makedirs(d, exist_ok=True)
        self.conn = sqlite3.connect(self.path, check_same_thread=False)
        log.info("成功連接到 L2 快取: %s", self.path)

    def init_schema(self):
        with self.conn:
            self.conn.execute(SCHEMA)

    def load_all_to_map(self) -> LockedDict:
        m = LockedDict()
        try:
            for wb, hb, sb, q, s in self.conn.execute(
                    "SELECT WIDTH_BUCKET, HEIGHT_BUCKET, SIZE_BUCKET, QUALITY, SCALE FROM LEARNED_PARAMS_CACHE"):
                m[SimilarityKey(int(wb), int(hb), int(sb))] = LearnedParams(float(np.float32(q)), float(s))
        except sqlite3.Error:
            log.exception("從 L2 快取載入時發生錯誤")  # the reference continues with what it has
        log.info("從 L2 快取載入 %d 筆學習參數到 L1", len(m))
        return m

    def save_all_from_map(self, m, batch_size: int = 1000) -> int:
        rows = [(k.width_bucket, k.height_bucket, k.size_bucket, float(np.float32(v.quality)), float(v.scale))
                for k, v in list(m.items())]
        if not rows:
            return 0
        try:
            with self.conn:  # one transaction; rolled back if any batch fails
                for i in range(0, len(rows), batch_size):
                    self.conn.executemany(
                        "INSERT OR REPLACE INTO LEARNED_PARAMS_CACHE "
                        "(WIDTH_BUCKET, HEIGHT_BUCKET, SIZE_BUCKET, QUALITY, SCALE) VALUES (?, ?, ?, ?, ?)",
                        rows[i:i + batch_size])
        except sqlite3.Error:
            log.exception("儲存 L1 快取至 L2 時發生錯誤，交易已回滾")
            return 0
        log.info("成功將 %d 筆 L1 快取資料寫回 L2", len(rows))
        return len(rows)

    def close(self):
        if self.conn is not None:
            self.conn.close()
            self.conn = None
