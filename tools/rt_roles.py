"""Which gf_bs_kernel launches of the round trip are GetPieces and which are
encodes (shared by prof_roundtrip.py, pmc_roundtrip.py, pmc_valu.py).

When the round trip's encode and GetPieces launch the same kernel instance on
the same grid (a plan choice: the encode of k + 2 rows takes KW = 4 today,
GetPieces of k rows the direct plan), the grid cannot tell them apart.  Order
does: GetPieces of a step starts (or is
dispatched) after that step's twin copy (copy_bitslice_*), and it is the
first launch of its grid to do so; the encodes are the rest (a pipelined
step's next encode starts beside the elimination, before the copy)."""


def get_ids(seq, grid_of, is_copy, key):
    """seq: launches in start (or dispatch) order; grid_of(x): the launch's
    grid or None if it is not a gf_bs_kernel launch; is_copy(x): a twin copy;
    key(x): an id.  Returns {(grid, ...)}: the ids of the GetPieces launches."""
    gets, armed = set(), False
    for x in seq:
        if is_copy(x):
            armed = True
        elif armed and grid_of(x) is not None:
            gets.add(key(x))
            armed = False
    return gets
