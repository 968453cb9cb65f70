import sys; sys.path.insert(0, "tools"); sys.path.insert(0, ".")
import stamps_rows as s
s.main("MOL", 115, 400)
s.main("MOL", 32, 1000)
s.main("MOL", 10, 1000)
