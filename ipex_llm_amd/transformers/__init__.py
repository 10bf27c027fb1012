"""HF-compatible model API (reference: ``SRC/transformers/__init__.py``)."""
from .low_bit_linear import LowBitLinear, DenseLinear, FP16Linear, BF16Linear, MatMulLowBit  # noqa: F401
from .model import (AutoModelForCausalLM, AutoModel, AutoModelForSpeechSeq2Seq,  # noqa: F401
                    AutoModelForSeq2SeqLM, AutoModelForSequenceClassification, AutoModelForMaskedLM,
                    AutoModelForQuestionAnswering, AutoModelForNextSentencePrediction,
                    AutoModelForMultipleChoice, AutoModelForTokenClassification, AutoModelForImageTextToText,
                    AutoModelForVision2Seq, save_low_bit)
from .convert import ggml_convert_low_bit  # noqa: F401
from .hybrid import convert_model_hybrid  # noqa: F401
