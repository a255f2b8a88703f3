"""Stand-in for recbole.model.abstract_recommender (only what RecBLR.py uses)."""
from torch import nn


class SequentialRecommender(nn.Module):
    def __init__(self, config, dataset):
        super().__init__()
        self.ITEM_ID = "item_id"
        self.ITEM_SEQ = "item_id_list"
        self.ITEM_SEQ_LEN = "item_length"
        self.POS_ITEM_ID = "item_id"
        self.NEG_ITEM_ID = "neg_item_id"
        self.max_seq_length = config["MAX_ITEM_LIST_LENGTH"]
        self.n_items = dataset.num("item_id")

    def gather_indexes(self, output, gather_index):
        idx = gather_index.view(-1, 1, 1).expand(-1, -1, output.shape[-1])
        return output.gather(dim=1, index=idx).squeeze(1)
