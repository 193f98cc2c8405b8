"""``H2OTwoDimTable`` (reference: h2o-py/h2o/two_dim_table.py): a titled table with a column header, column
types and row-major cell values; ``as_data_frame()`` gives pandas, ``t["col"]`` a column's values."""
from __future__ import annotations


class H2OTwoDimTable:
    def __init__(self, table_header=None, table_description=None, col_header=None, cell_values=None,
                 raw_cell_values=None, col_types=None, row_header=None, col_formats=None):
        self.table_header = table_header or ""
        self.table_description = table_description or ""
        self.col_header = list(col_header or [])
        self.cell_values = [list(r) for r in (cell_values if cell_values is not None else raw_cell_values or [])]
        self.col_types = list(col_types or [])
        self.row_header = row_header
        self.col_formats = col_formats

    @staticmethod
    def from_data_frame(df, table_header=None):
        return H2OTwoDimTable(table_header, col_header=list(df.columns), cell_values=df.values.tolist())

    def as_data_frame(self):
        import pandas as pd
        return pd.DataFrame(self.cell_values, columns=self.col_header or None)

    def __getitem__(self, item):
        if isinstance(item, (list, tuple)):
            return [self[i] for i in item]
        j = self.col_header.index(item) if isinstance(item, str) else int(item)
        return [r[j] for r in self.cell_values]

    def __len__(self):
        return len(self.cell_values)

    @property
    def nrows(self):
        return len(self.cell_values)

    @property
    def ncols(self):
        return len(self.col_header)

    def show(self, header=True):
        if header and self.table_header:
            print(self.table_header + (": " + self.table_description if self.table_description else ""))
        print(self.as_data_frame().to_string(index=False))

    def __repr__(self):
        return f"{self.table_header}\n{self.as_data_frame()}"
