"""Diagnostic: why a device string column gets materialized by `col = 'text'` (GPU box)."""
import os
import sys
import tempfile
import traceback

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import test_gpu_csv_strings as T  # noqa: E402
from net.jgp.labs.sparkdq4ml_amd import col  # noqa: E402
from net.jgp.labs.sparkdq4ml_amd.sql import table  # noqa: E402

orig = table.DeviceStringColumn.values.fget


def traced(self):
    if self._vals is None:
        print("MATERIALIZE n=%d dbuf=%s" % (self.n, self.dbuf is not None), flush=True)
        traceback.print_stack(limit=12)
    return orig(self)


table.DeviceStringColumn.values = property(traced, table.DeviceStringColumn.values.fset)
d = tempfile.mkdtemp()
p = os.path.join(d, "eq.csv")
open(p, "wb").write(T._mixed_csv(20_000, seed=4))
spark = T._session("0")
df = spark.read().option("inferSchema", "true").csv(p)
base = df._plan.table.columns[1]
print("base type", type(base).__name__, "dbuf", getattr(base, "dbuf", None) is not None, "opts", getattr(base, "opts", None))
got = [r[0] for r in df.filter(col("_c1") == "a").select("_c0").collect()]
print("rows", len(got), "materialized", base.materialized, flush=True)
