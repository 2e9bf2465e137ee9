"""MI355X-native drop-in for the reference's ``app`` package (hot path only).

Import surface mirrors Sabarna07-tech/Multimodal-RAG-for-Image-Text-Search:
``app.ml.embeddings``, ``app.ml.index_build``, ``app.ml.retrieve``,
``app.storage.lancedb_store``, ``app.cache``; the engine lives in
``app.vector_store`` (GPU flat index, C ABI ``include/mrag.h``) and
``app.retrieval`` (batched search + fusion).
"""
