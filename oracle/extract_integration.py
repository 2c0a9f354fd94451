"""Writes every ```c++ block of INTEGRATION.md, in document order, into one file (with #line
directives pointing back at the document), for oracle/integration_main.cpp to compile as
printed.  Test infrastructure: `make -C oracle integ` runs it; nothing in the product uses it.
Usage: python3 extract_integration.py INTEGRATION.md out.inc"""
import os
import sys


def blocks(md: str):
    out, cur, start = [], None, 0
    for i, line in enumerate(md.splitlines(), 1):
        if cur is None and line.strip() == "```c++":
            cur, start = [], i + 1
        elif cur is not None and line.strip() == "```":
            out.append((start, cur))
            cur = None
        elif cur is not None:
            cur.append(line)
    if cur is not None:
        raise SystemExit("unterminated c++ block")
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    bl = blocks(open(src).read())
    if not bl:
        raise SystemExit(f"no c++ blocks in {src}")
    with open(dst, "w") as f:
        f.write(f"// generated from {src} by oracle/extract_integration.py: do not edit\n")
        for start, lines in bl:
            f.write(f"#line {start} \"{os.path.basename(src)}\"\n")
            f.write("\n".join(lines) + "\n")
    print(f"{len(bl)} blocks -> {dst}")


if __name__ == "__main__":
    main()
