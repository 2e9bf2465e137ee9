"""CPU oracle for the hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import anything from this package, and only as the checker / the timed CPU
baseline — never as part of the product path (which fails loudly without
``libmrag.so``).

Contents (each function cites the reference file:line it restates):
  knn.py        exact flat cosine top-k (lancedb flat scan, app/storage/lancedb_store.py:103-139)
  normalize.py  the two reference normalisers (app/ml/embeddings.py:46-49, lancedb_store.py:63-69)
  fusion.py     z-score fusion (app/ml/retrieve.py:158-195)
  models.py     CLIP ViT-B/32 / CLIP text / MiniLM-L6 forward on torch-CPU fp32
  gen_golden.py generator of tests/golden/* (imports the reference itself, with stubs)

Pinning: see DESIGN.md §5 (which fixtures pin which function).
"""
