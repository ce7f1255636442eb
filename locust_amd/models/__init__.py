"""MapReduce jobs ("models").  WordCount is the reference's job (README.md:26)."""
from .wordcount import Engine, WordCount, run_multi, wordcount_file, wordcount_text

__all__ = ["Engine", "WordCount", "run_multi", "wordcount_file", "wordcount_text"]
