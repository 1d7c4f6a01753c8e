"""MI355X-native Batcher for the streaming NLP data loader (andywag/streaming_data_loader).

The Batcher's per-record tokenize-and-mask path (raw UTF-8 -> WordPiece ids ->
MLM mask / CLM labels -> packed [B,S] int32) runs as hand-written gfx950 HIP
kernels behind the C ABI in include/sdl_batcher.h (libsdl_batcher.so).  This
package is the Python host mirror of the reference's Batcher interface.
"""
from .batcher import (Batcher, BatchConfig, DataSet, GenTokenizer, Gpt, Label, Mask, ModelType,  # noqa: F401
                      MultiLabel, ProviderChannel, ShardedGenTokenizer, SimpleBatcher, SimpleData, SimpleTransport, SingleClass, Span,
                      TaskType,
                      TokenizerConfig, TrainingConfig, create_batch, create_batch_drained, get_case,
                      get_mask_length)
from .native import SDLError  # noqa: F401
