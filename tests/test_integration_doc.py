"""CPU: INTEGRATION.md §3 names every entry point of the product header
(include/beatrice_gpu.h), and its table names nothing the header does not declare — the
drop-in contract a maintainer binds is exactly what the document lists."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(path):
    src = re.sub(r"/\*.*?\*/", "", open(path).read(), flags=re.S)
    return set(re.findall(r"^\s*[A-Za-z_][\w\s\*]*?\b(bt_[a-z0-9_]+)\s*\(", src, flags=re.M))


def test_integration_table_matches_product_header():
    product = _declared(os.path.join(ROOT, "include", "beatrice_gpu.h"))
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    start = doc.index("**Every entry point of `include/beatrice_gpu.h`**")
    table = doc[start:doc.index("\n\n", doc.index("| Entry points |", start))]
    named = set()
    for line in table.splitlines():
        if line.startswith("| `bt_"):
            named |= set(re.findall(r"`(bt_[a-z0-9_]+)`", line.split("|")[1]))
    assert product - named == set(), f"product entry points the table does not name: {sorted(product - named)}"
    assert named - product == set(), f"table names that the product header does not declare: {sorted(named - product)}"
    assert f"**Every entry point of `include/beatrice_gpu.h`** ({len(product)};" in doc
