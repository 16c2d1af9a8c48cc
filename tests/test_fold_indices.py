"""CPU check of the folded BN finalize's prologue indexing (hgk_conv.hip, conv_fwd_body FOLDK): for
every input-channel count a launch admits (hgk_conv_fold_ok: Cin <= 256) and every partial-row
count (<= 32, multiple of 4), each of the NT = 256 threads reads only its channel's partial rows
and exchanges with a thread of the workgroup — the same expressions as the kernel. (A first
version let the threads past 2 * Cin read past the partials when Cin < 128.)"""

NT, FOLD_ROWS = 256, 32
FV = FOLD_ROWS // 4


def _thread_reads(Cin, rows, tid):
    nv = rows >> 2
    ftwo = 2 * Cin <= NT
    fstep = 2 if ftwo else 1
    fh = 1 if (ftwo and tid >= Cin) else 0
    fc = min(tid - Cin if fh else tid, Cin - 1)
    reads = []
    for j in range(FV):
        jj = min(j * fstep + fh, nv - 1)
        for k in range(3):
            reads.append(fc * 3 * rows + (k * nv + jj) * 4)  # float4 at this float index
    partner = (tid - Cin if fh else tid + Cin) if ftwo else None
    return fc, reads, partner


def test_fold_prologue_reads_stay_in_the_partials():
    for Cin in (64, 96, 128, 192, 256):
        for rows in range(4, FOLD_ROWS + 1, 4):
            for tid in range(NT):
                fc, reads, partner = _thread_reads(Cin, rows, tid)
                assert 0 <= fc < Cin
                assert all(0 <= r and r + 3 < Cin * 3 * rows for r in reads), (Cin, rows, tid)
                if partner is not None:
                    assert 0 <= partner < NT


def test_fold_prologue_pairs_cover_every_row_once():
    """two threads per channel (Cin <= 128) take alternate row quads: together every quad once"""
    for Cin in (64, 128):
        for rows in range(4, FOLD_ROWS + 1, 4):
            nv = rows >> 2
            for c in range(Cin):
                seen = []
                for tid in (c, c + Cin):
                    fh = 1 if tid >= Cin else 0
                    myq = (nv - fh + 1) // 2
                    seen += [j * 2 + fh for j in range(myq)]
                assert sorted(seen) == list(range(nv)), (Cin, rows, c)
