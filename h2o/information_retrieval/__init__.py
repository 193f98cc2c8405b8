"""``h2o.information_retrieval`` (reference: h2o-py/h2o/information_retrieval/tf_idf.py)."""


def tf_idf(frame, document_id_col, text_col, preprocess=True, case_sensitive=True):
    """TF-IDF of the words of ``text_col`` per document of ``document_id_col`` (columns DocID, Word, TF, IDF,
    TF-IDF); ``preprocess`` splits the text into words first."""
    from llama_github_io_amd.frame_ops import tf_idf as _tf_idf
    return _tf_idf(frame, document_id_col, text_col, preprocess, case_sensitive)


__all__ = ["tf_idf"]
