"""Modeling library (reference runtime/ai/modeling/): histogram gradient-boosted trees
(``gbdt``, the XGBoost workload), GraphSAGE (``graph_sage``) and transfer learning
(``transfer_learning``), all on the MI355X op library."""
