import os, sys; sys.path.insert(0, "tools"); sys.path.insert(0, ".")
import stamps_rows as s
for g in ("1", "2"):
    os.environ["WRNN_ROW_GROUPS"] = g
    print("groups", g)
    s.main("MOL", 2, 1000)
    s.main("MOL", 4, 1000)
    s.main("RAW", 10, 1000)
