"""The oracle statement of what each raster evaluation form of libuampath computes (test
infrastructure): K2h (the default for large generated batches: K2g's grouped raster sums, the
geometry terms in the similarity form) -> orc_eval_generated_h; K2g -> orc_eval_paths_g; every
other form -> the reference's sequential order (orc_eval_paths)."""


def raster_ref(oracle_mod, orc, kernel, group, pairs, ut, rd, rec, want_cells=False):
    if kernel.startswith("K2h"):
        return orc.eval_generated_h(pairs, ut, rdesc=rd, rec=rec, group=group,
                                    want_cells=want_cells)
    return orc.eval_paths(oracle_mod.gen_paths(pairs, ut), mode="raster", rdesc=rd, rec=rec,
                          group=group if kernel == "K2g+pack" else 0, want_cells=want_cells)
