"""Model / serving constants of the reference (``src/config.py:17-50``,
``app/src/config.py:22-59``) that the engine and its callers need."""
from dataclasses import dataclass


@dataclass(frozen=True)
class Config:
    img_h: int = 96               # serving / training resize target (app/src/config.py:23-24)
    img_w: int = 320
    d_model: int = 256
    nhead: int = 8
    num_decoder_layers: int = 8
    dim_feedforward: int = 512
    dropout: float = 0.2          # app/src/config.py:29 (training only; reported by /model/info)
    max_seq_len: int = 150        # greedy loop bound and positional-table rows
    sos_token: str = "<sos>"
    eos_token: str = "<eos>"
    pad_token: str = "<pad>"
    unk_token: str = "<unk>"
    max_file_size: int = 10 * 1024 * 1024                     # app/src/config.py:58
    allowed_extensions: tuple = (".jpg", ".jpeg", ".png", ".bmp", ".tiff", ".webp")
    max_batch_images: int = 10                                # app/src/models.py:34
    api_version: str = "1.0.0"                                # app/src/config.py:18

    @property
    def special_tokens(self):                                 # app/src/config.py:47
        return [self.pad_token, self.sos_token, self.eos_token, self.unk_token]


config = Config()
