"""Py/xshard/utils.py helpers."""


def chunk(lst, n):
    """Split ``lst`` into ``n`` nearly equal consecutive chunks."""
    size, rem = divmod(len(lst), n)
    out, i = [], 0
    for k in range(n):
        j = i + size + (1 if k < rem else 0)
        out.append(lst[i:j])
        i = j
    return out


def flatten(list_of_list):
    return [x for sub in list_of_list for x in sub]
