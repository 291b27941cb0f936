# timing bound only (WRONG sums): the grid kernel without the 1/|B'| table read
s|const double invb_new = p.g.invb\[bnodes + plus - minus\];|const double invb_new = invb + (double)(plus - minus);|
