"""Child order of a reference MetricsTree node, restated.

The reference keeps children in a java.util.concurrent.ConcurrentHashMap and
exposes them as `trees.toMap` (MetricsTree.scala:44-45): a Scala 2.12 immutable
Map built from the ConcurrentHashMap's iteration order.  Every exporter walks
`tree.children` in that order (PrometheusTelemeter.scala:128, InfluxDbTelemeter.scala:79,
AdminMetricsExportTelemeter.scala:131,144), so exact output order depends on it
(e.g. `{"bass":1,"bas":1}` at AdminMetricsExportTelemeterTest.scala:111).

  * <= 4 children: scala.collection.immutable.Map1..Map4 keep the insertion
    order of the builder, i.e. the ConcurrentHashMap iteration order: table bins
    in index order (index = spread(String.hashCode) & (n - 1), table of 16 bins
    doubling at 3/4 load), list order inside a bin, with the list split of a
    resize (JDK 8 ConcurrentHashMap.transfer: the trailing run keeps its order,
    the nodes before it are prepended).
  * >= 5 children: scala.collection.immutable.HashMap (hash trie): iteration is
    by the 5-bit chunks of improve(hashCode), lowest chunk first.
Bins that would become red-black trees (>= 8 colliding keys) are not modelled.
Pinned against the key order of the reference's tree-mode fixture
(tests/golden/metrics_key_order.json).
"""
from __future__ import annotations

from typing import Iterable, List

_M32 = 0xFFFFFFFF


def _i32(x: int) -> int:
    x &= _M32
    return x - (1 << 32) if x & 0x80000000 else x


def java_string_hash(s: str) -> int:
    """java.lang.String.hashCode over UTF-16 code units (signed 32-bit)."""
    h = 0
    b = s.encode("utf-16-le", "surrogatepass")
    for i in range(0, len(b), 2):
        h = (31 * h + (b[i] | (b[i + 1] << 8))) & _M32
    return _i32(h)


def _spread(h: int) -> int:
    h &= _M32
    return (h ^ (h >> 16)) & 0x7FFFFFFF


def chm_order(keys_in_insertion_order: Iterable[str]) -> List[str]:
    """Iteration order of a JDK 8 ConcurrentHashMap after putting the keys in order."""
    n = 16
    size_ctl = n - (n >> 2)
    table: List[List[tuple]] = [[] for _ in range(n)]
    count = 0
    for k in keys_in_insertion_order:
        h = _spread(java_string_hash(k))
        b = table[h & (n - 1)]
        if any(kk == k for _, kk in b):
            continue
        b.append((h, k))
        count += 1
        if count >= size_ctl:  # addCount -> transfer to a table twice as big
            nt: List[List[tuple]] = [[] for _ in range(2 * n)]
            for i, bin_ in enumerate(table):
                if not bin_:
                    continue
                run_bit = bin_[0][0] & n
                last = 0
                for j in range(1, len(bin_)):
                    bb = bin_[j][0] & n
                    if bb != run_bit:
                        run_bit, last = bb, j
                lo = bin_[last:] if run_bit == 0 else []
                hi = bin_[last:] if run_bit != 0 else []
                for node in bin_[:last]:  # prepended, one by one
                    if node[0] & n == 0:
                        lo = [node] + lo
                    else:
                        hi = [node] + hi
                nt[i], nt[i + n] = lo, hi
            size_ctl = (n << 1) - (n >> 1)
            n *= 2
            table = nt
    return [k for bin_ in table for _, k in bin_]


def scala_improve(hcode: int) -> int:
    """scala.collection.immutable.HashMap.improve (2.12)."""
    h = (hcode + ~(hcode << 9)) & _M32
    h ^= h >> 14
    h = (h + (h << 4)) & _M32
    return (h ^ (h >> 10)) & _M32


def _trie_key(k: str):
    h = scala_improve(java_string_hash(k))
    return tuple((h >> (5 * lvl)) & 31 for lvl in range(7))


def reference_child_order(keys_in_insertion_order: Iterable[str]) -> List[str]:
    """Order of `ConcurrentHashMap(keys).asScala.toMap` iteration."""
    keys = chm_order(keys_in_insertion_order)
    if len(keys) <= 4:
        return keys
    return sorted(keys, key=_trie_key)
